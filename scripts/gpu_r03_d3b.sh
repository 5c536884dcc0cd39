#!/bin/bash
# byte-run pre hash: update parity tests, then d3 DELTA A/B (HF3FS_CRC_PRE_RUNS) in alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "update or cpp" --timeout 180 --timeout-method thread > $O/upd_tests2.log 2>&1; rc=$?
tail -3 $O/upd_tests2.log; [ $rc -eq 0 ] || exit $rc
export D3_MODES=${D3_MODES:-delta} D3_AB=0 SUITE_CPU=0
for rep in 1 2 3; do
for v in 1 0; do
  HF3FS_CRC_PRE_RUNS=$v timeout -k 10 120 python3 tests/bench_suite.py d3 > $O/d3_runs$v.log 2>&1 || exit $?
  echo "runs=$v $(tail -1 $O/d3_runs$v.log | grep -o '"delta": {[^}]*}')"
done
done
