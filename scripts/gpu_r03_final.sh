#!/bin/bash
# Round-3 evidence on the current build: every -m gpu test, smoke, the driver's bench line +
# its rocprofv3 trace and PMC passes, the d3 kernel trace, and the full suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/gpu_tests_final.log 2>&1; rc=$?
tail -2 $O/gpu_tests_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final.log 2>&1 || exit $?
tail -1 $O/smoke_final.log
bash scripts/gpu_prof_round.sh || exit $?
SUITE_CPU=${SUITE_CPU:-1} timeout -k 10 900 python3 -u tests/bench_suite.py > $O/suite_final.log 2>&1 || { tail -5 $O/suite_final.log; exit 1; }
grep '^{' $O/suite_final.log | cut -c1-200
