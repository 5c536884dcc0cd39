#!/bin/bash
# Full GPU check: every -m gpu test (service mode included), smoke, bench.py. Stops at the first crash-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread
run smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python -u bench.py
