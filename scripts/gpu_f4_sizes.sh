#!/bin/bash
# f4 per-size-class timing (one size at a time): where the per-frame overhead sits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for cfg in "64 1000000" "256 1000000" "1024 1000000" "4096 500000" "16384 200000" "64,256,1024,4096,16384 1000000"; do
  set -- $cfg
  F4_SIZES=$1 F4_N=$2 timeout -k 10 200 python -u tests/bench_suite.py f4 > gpurun_out/f4s.log 2>&1; rc=$?
  echo "sizes=$1 n=$2 rc=$rc $(tail -1 gpurun_out/f4s.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*\|"frames_per_s": [0-9]*\|"mismatch_set_exact": [a-z]*' | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
