#!/bin/bash
# Round measurement: every GPU test, smoke, the default bench line, the bench
# suite (d3 d4 d5 f2 f3 f4), the randomized soak against the oracle (SOAK_SECONDS,
# default 240), then the rocprofv3 kernel trace + PMC passes of bench.py.  Stops at the
# first crash-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run tests 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread
run smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python -u bench.py
run suite 900 python -u tests/bench_suite.py
run soak $(( ${SOAK_SECONDS:-240} + 120 )) python -u tests/soak.py ${SOAK_SECONDS:-240}
bash scripts/gpu_profile.sh; echo "profile rc=$?"
