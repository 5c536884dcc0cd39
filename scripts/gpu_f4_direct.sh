#!/bin/bash
# record jobs on the DIRECT instantiation: f4 mix and size classes, pipe A/B; d5; update parity; frame/scrub/read tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_aux.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/t.log)"; [ $rc -ne 0 ] && exit $rc
for cfg in "mix 1000000 d 1" "mix 1000000 0 1" "mix 1000000 d 0" "64 1000000 d 1" "64 1000000 0 1" "16384 200000 d 1" "16384 200000 0 1"; do
  set -- $cfg
  if [ "$3" = "d" ]; then unset HF3FS_CRC_PIPE; else export HF3FS_CRC_PIPE=$3; fi
  if [ "$1" = "mix" ]; then SZ=64,256,1024,4096,16384; else SZ=$1; fi
  HF3FS_CRC_RECORD_DIRECT=$4 F4_SIZES=$SZ F4_N=$2 timeout -k 10 200 python -u tests/bench_suite.py f4 > gpurun_out/f4s.log 2>&1; rc=$?
  echo "sizes=$1 pipe=$3 direct=$4 rc=$rc $(tail -1 gpurun_out/f4s.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*\|"mismatch_set_exact": [a-z]*' | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
done
unset HF3FS_CRC_PIPE
timeout -k 10 200 python -u tests/bench_suite.py d5 > gpurun_out/d5.log 2>&1; echo "d5 rc=$? $(tail -1 gpurun_out/d5.log | grep -o '"gbs": [0-9.]*')"
