#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03; mkdir -p $O; rm -f $O/first_call.log
for args in "1" "1" "0" "1 warm" "1 grow" "1 ref200" "1 ref200" "0 ref5"; do
  echo "== $args" >> $O/first_call.log
  HF3FS_CRC_DEBUG=1 timeout -k 5 60 ./build/probe_first_call $args >> $O/first_call.log 2>&1 || exit $?
done
timeout -k 5 120 ./tests/cpp/test_checksuminfo > $O/cpp_dropin.log 2>&1; echo "cpp rc=$?" >> $O/first_call.log
grep -E "mode=|staged|retry|FAILED|ALL OK" $O/cpp_dropin.log | head -8 >> $O/first_call.log
cat $O/first_call.log
