#!/bin/bash
# Current build: f4 kernel trace (mix), suite legs d3/d5/f4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
SUITE_CPU=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/f4trace2 -o run --output-format csv -- python3 -u tests/bench_suite.py f4 > $O/f4trace2.log 2>&1 || { tail -5 $O/f4trace2.log; exit 1; }
echo "== f4 traced $(grep '^{' $O/f4trace2.log | grep -o '"ms_per_batch": [0-9.]*')"
python3 scripts/kstats.py $O/f4trace2 8
SUITE_CPU=0 timeout -k 10 400 python3 -u tests/bench_suite.py ${LEGS:-d3 d5 f4} > $O/suite_state.log 2>&1 || { tail -5 $O/suite_state.log; exit 1; }
grep '^{' $O/suite_state.log | cut -c1-330
