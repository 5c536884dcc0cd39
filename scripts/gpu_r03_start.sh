#!/bin/bash
# Session start on the GPU: every -m gpu test, smoke, bench, then the C++ drop-in test in
# fresh processes and the first-call probe (the first-DELTA-call report).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-600
bash scripts/gpu_r03_cpprep.sh 8 || exit $?
bash scripts/gpu_r03_first.sh
