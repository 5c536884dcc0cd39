#!/bin/bash
# Every -m gpu test on the current build, then the C++ drop-in test in N fresh processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r03_cpprep.sh ${CPPREP:-32} | tail -3
echo "cpp drop-in failed: $(grep -c 'rc=1' $O/cpprep.log) / $(grep -c '^run' $O/cpprep.log)"
