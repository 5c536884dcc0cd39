#!/bin/bash
# single-read DELTA pipeline: update parity (all pipelines), then the d3 A/B (default = single vs unfused vs fused).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "update" --timeout 180 --timeout-method thread > gpurun_out/upd_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/upd_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
D3_MODES=delta timeout -k 10 300 python -u tests/bench_suite.py d3 > gpurun_out/d3.log 2>&1; rc=$?
echo "d3 rc=$rc"; tail -1 gpurun_out/d3.log | cut -c1-1500
