#!/bin/bash
# d3 apply-piece A/B: update parity tests, then d3 (delta + reference) under
# different piece settings, then a per-kernel trace of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
run upd_tests 300 python -u -m pytest tests/test_gpu_parity.py -k update -x -q --timeout 120 --timeout-method thread
export D3_AB=0
run d3_p8 200 env HF3FS_CRC_APPLY_PIECES=8 python3 tests/bench_suite.py d3
run d3_p1 200 env HF3FS_CRC_APPLY_PIECES=1 HF3FS_CRC_APPLY_MIN_KIB=1048576 python3 tests/bench_suite.py d3
run d3_p4 200 env HF3FS_CRC_APPLY_PIECES=4 python3 tests/bench_suite.py d3
run d3_p16 200 env HF3FS_CRC_APPLY_PIECES=16 HF3FS_CRC_APPLY_MIN_KIB=32 python3 tests/bench_suite.py d3
run d3_ref_unfused 200 env HF3FS_CRC_UPDATE_UNFUSED=1 D3_MODES=reference python3 tests/bench_suite.py d3
run d3_seg128 200 env HF3FS_CRC_SEG_KIB=128 D3_MODES=delta python3 tests/bench_suite.py d3
mkdir -p gpurun_out/p3e
export D3_MODES=delta
run prof_d3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p3e -o run --output-format csv -- python3 tests/bench_suite.py d3
echo done
