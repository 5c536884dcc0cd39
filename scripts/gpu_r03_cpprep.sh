#!/bin/bash
# The C++ drop-in test in fresh processes (the round-1/3 first-DELTA-call report).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03; mkdir -p $O; rm -f $O/cpprep.log
N=${1:-16}
for i in $(seq 1 $N); do
  timeout -k 5 120 ./tests/cpp/test_checksuminfo > $O/cpprep_$i.log 2>&1; rc=$?
  echo "run $i rc=$rc $(tail -1 $O/cpprep_$i.log)" >> $O/cpprep.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || break
  [ $rc -eq 0 ] && rm -f $O/cpprep_$i.log
done
cat $O/cpprep.log
grep -h -A4 "mode=" $O/cpprep_*.log 2>/dev/null | head -40
