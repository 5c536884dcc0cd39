#!/bin/bash
# tests + suite (no profile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run tests 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run suite 900 python -u tests/bench_suite.py ${SUITE:-d3 d5}
