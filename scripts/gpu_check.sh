#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench. Stops at the first crash-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -3 gpurun_out/smoke.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 > gpurun_out/bench.log 2>&1
rc3=$?; echo "bench rc=$rc3"; tail -3 gpurun_out/bench.log
exit $(( rc | rc2 | rc3 ))
