#!/bin/bash
# Kernel trace of the suite's d5 leg (which kernels hold the time per batch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
SUITE_CPU=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d5trace -o run --output-format csv -- python3 -u tests/bench_suite.py d5 > $O/d5trace.log 2>&1 || { tail -5 $O/d5trace.log; exit 1; }
grep '^{' $O/d5trace.log | cut -c1-250
python3 scripts/kstats.py $O/d5trace 10
