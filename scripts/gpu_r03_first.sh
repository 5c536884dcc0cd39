#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03; mkdir -p $O
for args in "1" "1" "0" "1 warm" "0 warm"; do
  HF3FS_CRC_DEBUG=1 timeout -k 5 60 ./build/probe_first_call $args >> $O/first_call.log 2>&1 || exit $?
done
cat $O/first_call.log
