#!/bin/bash
# update pipeline: parity tests (fused + unfused), C++ drop-in, d3 A/B bench. Stops at the first crash-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run upd_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_dropin.py tests/test_file_digest.py -v --timeout 120 --timeout-method thread -k "update or dropin or combine or digest"
run d3 400 python -u tests/bench_suite.py d3
