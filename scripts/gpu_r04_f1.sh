#!/bin/bash
# Round 4, measurement pass 1: the GPU suite, smoke, the C++ drop-in test in 24 fresh processes
# (the incident's reproducer) with the self-check record, the default bench line, and bench.py's
# rocprofv3 kernel trace + PMC passes.
set -eo pipefail
O=gpurun_out/r04/f1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
fails=0
for k in $(seq 1 24); do
  rc=0; timeout -k 10 120 tests/cpp/test_checksuminfo > $O/cpp_$k.log 2>&1 || rc=$?
  if [ $rc -ge 124 ]; then echo "cpp run $k ended with $rc: stopping"; exit $rc; fi
  if [ $rc -ne 0 ]; then fails=$((fails+1)); fi
done
echo "cpp drop-in fresh processes: 24 runs, $fails failed" | tee $O/cpp_repeat.txt
grep -h "ALL OK\|FAIL" $O/cpp_*.log | sort | uniq -c >> $O/cpp_repeat.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
bash scripts/gpu_profile.sh
cp -r gpurun_out/prof $O/prof
echo done
