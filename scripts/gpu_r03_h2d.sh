#!/bin/bash
# d4 streamed-H2D probe + the suite's d4 leg and bench.py's h2d leg, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 300 python3 -u scripts/d4_h2d_probe.py > $O/h2d_probe.log 2>&1 || { tail -5 $O/h2d_probe.log; exit 1; }
cat $O/h2d_probe.log
SUITE_CPU=0 timeout -k 10 300 python3 -u tests/bench_suite.py d4 > $O/h2d_suite.log 2>&1 || exit $?
tail -1 $O/h2d_suite.log | cut -c1-400
timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/h2d_bench.log 2>&1 || exit $?
tail -1 $O/h2d_bench.log | grep -o '"pinned_h2d": {[^}]*}'
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/h2dtrace -o run --output-format csv -- python3 scripts/d4_h2d_probe.py > $O/h2dtrace.log 2>&1 || exit $?
echo traced
