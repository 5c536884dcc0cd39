#!/bin/bash
# Stale-payload investigation: the deterministic pageable-staging
# pattern, then the stress matrix over staging variants + the library-free probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tests/cpp/test_staging > gpurun_out/staging_det.log 2>&1; rc=$?
echo "det rc=$rc"; tail -2 gpurun_out/staging_det.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 ./tests/cpp/test_staging --stress ${STRESS:-300} > gpurun_out/staging_stress.log 2>&1; rc=$?
echo "stress rc=$rc"; tail -2 gpurun_out/staging_stress.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/tests.log
