#!/bin/bash
# f4 overhead diagnosis: alignment and cross-task prefetch, per size class.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for cfg in "64 1000000 0 d" "64 1000000 1 d" "64 1000000 0 0" "16384 200000 0 d" "16384 200000 1 d" "16384 200000 0 0" "4096 500000 1 d"; do
  set -- $cfg
  if [ "$4" = "d" ]; then unset HF3FS_CRC_PIPE; else export HF3FS_CRC_PIPE=$4; fi
  F4_ALIGN=$3 F4_SIZES=$1 F4_N=$2 timeout -k 10 200 python -u tests/bench_suite.py f4 > gpurun_out/f4s.log 2>&1; rc=$?
  echo "sizes=$1 align=$3 pipe=$4 rc=$rc $(tail -1 gpurun_out/f4s.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*\|"frames_per_s": [0-9]*\|"mismatch_set_exact": [a-z]*' | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
