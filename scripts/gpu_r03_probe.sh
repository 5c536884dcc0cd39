#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 180 ./build/probe_copy ${1:-5} ${2:-bodies,mall,sub} > $O/probe_copy2.log 2>&1; rc=$?
cat $O/probe_copy2.log; exit $rc
