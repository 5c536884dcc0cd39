#!/bin/bash
# f3/f4 GPU tests + bench legs. Stops at the first crash-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run aux_tests 300 python -u -m pytest tests/test_gpu_aux.py -v --timeout 120 --timeout-method thread
run aux_bench 400 python -u tests/bench_suite.py f3 f4
