#!/bin/bash
# Round 3, first GPU call: the apply-copy probe, then the d3 DELTA leg under
# rocprofv3 (kernel trace + stats) and two PMC passes (FETCH_SIZE, WRITE_SIZE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 180 ./build/probe_copy 5 > $O/probe_copy.log 2>&1 || { echo "probe rc=$?"; exit 1; }
cat $O/probe_copy.log
export D3_MODES=delta D3_AB=0 SUITE_CPU=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/d3trace -o run --output-format csv -- python3 tests/bench_suite.py d3 > $O/d3trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
tail -1 $O/d3trace.log | cut -c1-600
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/d3fetch -o run --output-format csv -- python3 tests/bench_suite.py d3 > $O/d3fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/d3write -o run --output-format csv -- python3 tests/bench_suite.py d3 > $O/d3write.log 2>&1 || { echo "write rc=$?"; exit 1; }
python3 scripts/pmc_summary.py $O | grep -E "==|k_" | cut -c1-300
echo done
