#!/bin/bash
# The C++ drop-in test in fresh processes: default vs code objects loaded at startup
# (HIP_ENABLE_DEFERRED_LOADING=0), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03; mkdir -p $O; rm -f $O/lazy.log
for i in $(seq 1 ${REPS:-16}); do
  for v in 1 0; do
    HIP_ENABLE_DEFERRED_LOADING=$v timeout -k 5 120 ./tests/cpp/test_checksuminfo > $O/lazy_run.log 2>&1; rc=$?
    echo "deferred=$v run $i rc=$rc $(tail -1 $O/lazy_run.log)" >> $O/lazy.log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || { cat $O/lazy.log; exit $rc; }
    [ $rc -eq 1 ] && grep -m1 -A1 "mode=" $O/lazy_run.log >> $O/lazy.log
  done
done
cat $O/lazy.log
echo "deferred=1 failed: $(grep -c 'deferred=1 .*rc=1' $O/lazy.log) / $(grep -c 'deferred=1 ' $O/lazy.log)"
echo "deferred=0 failed: $(grep -c 'deferred=0 .*rc=1' $O/lazy.log) / $(grep -c 'deferred=0 ' $O/lazy.log)"
