#!/bin/bash
# round 6: the -m gpu suite, smoke, bench.py, the d3 trace (checkpoint of a build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r06_gpu_tests.log 2>&1 || exit $?
bash scripts/gpu_steps.sh smoke bench profd3
