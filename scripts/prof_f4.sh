#!/bin/bash
# frame parity, then per-kernel times of f4 (stream path) per size class and the mix
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/pf4
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_aux.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/t.log)"; [ $rc -ne 0 ] && exit $rc
# PROF_CFGS: "sizes:n:name" entries separated by spaces
PROF_CFGS=${PROF_CFGS:-"1024:1000000:k1 16384:200000:k16 4096:500000:k4 64:1000000:b64 64,256,1024,4096,16384:1000000:mix"}
for cfg in $PROF_CFGS; do
  IFS=: read -r s1 s2 s3 <<< "$cfg"; set -- "$s1" "$s2" "$s3"
  F4_SIZES=$1 F4_N=$2 timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/pf4/$3 -o run -- python3 -u tests/bench_suite.py f4 > gpurun_out/pf4/$3.log 2>&1; rc=$?
  echo "cfg=$3 rc=$rc $(tail -1 gpurun_out/pf4/$3.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*\|"mismatch_set_exact": [a-z]*' | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
exit 0
