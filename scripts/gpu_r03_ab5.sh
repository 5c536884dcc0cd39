#!/bin/bash
# d5 balanced-run pipeline A/B (base vs runpipe, one process) after the staging probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
[ -n "$STG" ] && { bash scripts/gpu_r03_staging.sh $STG || exit $?; }
AB_LIBS="${AB_LIBS:-base runpipe}" AB_CASES="${AB_CASES:-d5 d5u4 d5u64 d2}" timeout -k 10 300 python3 -u scripts/ab_ranges_inproc.py > $O/ab5.log 2>&1; rc=$?
cat $O/ab5.log; exit $rc
