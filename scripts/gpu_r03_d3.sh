#!/bin/bash
# d3 rework check: update parity tests, then the d3 DELTA leg A/B (apply order) and a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "update or cpp" --timeout 180 --timeout-method thread > $O/upd_tests.log 2>&1; rc=$?
tail -3 $O/upd_tests.log; [ $rc -eq 0 ] || exit $rc
export D3_MODES=${D3_MODES:-delta} D3_AB=0 SUITE_CPU=0
for rep in 1 2; do
for rev in 0 1; do
  HF3FS_CRC_APPLY_REVERSE=$rev timeout -k 10 120 python3 tests/bench_suite.py d3 > $O/d3_rev$rev.log 2>&1 || exit $?
  echo "rev=$rev $(tail -1 $O/d3_rev$rev.log | grep -o '"delta": {[^}]*}')"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d3trace2 -o run --output-format csv -- python3 tests/bench_suite.py d3 > $O/d3trace2.log 2>&1 || exit $?
echo traced
