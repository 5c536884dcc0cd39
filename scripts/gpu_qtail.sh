#!/bin/bash
# hash_grid leftover-block queueing: parity, f4 size classes, d5, d4 and the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_aux.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/t.log)"; [ $rc -ne 0 ] && exit $rc
for cfg in "64 1000000" "256 1000000" "1024 1000000" "4096 500000" "16384 200000" "64,256,1024,4096,16384 1000000"; do
  set -- $cfg
  F4_SIZES=$1 F4_N=$2 timeout -k 10 200 python -u tests/bench_suite.py f4 > gpurun_out/f4s.log 2>&1; rc=$?
  echo "f4 sizes=$1 rc=$rc $(tail -1 gpurun_out/f4s.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*\|"mismatch_set_exact": [a-z]*' | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
done
for c in d5 d4; do
  timeout -k 10 300 python -u tests/bench_suite.py $c > gpurun_out/$c.log 2>&1; rc=$?
  echo "$c rc=$rc $(tail -1 gpurun_out/$c.log | grep -o '"gbs": [0-9.]*\|"bit_exact[a-z_]*": [a-z]*' | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/b.log 2>&1; rc=$?
echo "bench rc=$rc $(tail -1 gpurun_out/b.log | cut -c1-400)"
exit $rc
