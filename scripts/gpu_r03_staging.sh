#!/bin/bash
# Small pageable H2D after an async memset of another buffer (probe_staging), then the C++
# drop-in test in fresh processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 240 ./build/probe_staging ${1:-50000} > $O/probe_staging.log 2>&1; rc=$?
cat $O/probe_staging.log; [ $rc -eq 0 ] || exit $rc
