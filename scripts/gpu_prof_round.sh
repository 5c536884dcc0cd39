#!/bin/bash
# Round-end evidence: the driver's default bench command (JSON line kept) and its
# rocprofv3 kernel trace + PMC passes, then the d3 per-kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-400
bash scripts/gpu_profile.sh || exit $?
mkdir -p gpurun_out/p3
D3_AB=0 D3_MODES=delta,reference timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p3 -o run --output-format csv -- python3 tests/bench_suite.py d3 > gpurun_out/p3.log 2>&1 || exit $?
tail -1 gpurun_out/p3.log | cut -c1-300
