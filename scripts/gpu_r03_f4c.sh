#!/bin/bash
# Frame tests + the suite's f4 leg on the current build, then the C++ drop-in test in fresh
# processes with the library's debug dump (HF3FS_CRC_DEBUG: pre/post hashes read back after
# every update call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py -k "frame or Frame" -m gpu -x -q --timeout 120 --timeout-method thread > $O/frame_tests.log 2>&1; rc=$?
tail -3 $O/frame_tests.log; [ $rc -eq 0 ] || exit $rc
SUITE_CPU=0 timeout -k 10 300 python3 -u tests/bench_suite.py f4 > $O/suite_f4.log 2>&1 || { tail -5 $O/suite_f4.log; exit 1; }
grep '^{' $O/suite_f4.log | cut -c1-400
HF3FS_CRC_DEBUG=1 bash scripts/gpu_r03_cpprep.sh ${CPPREP:-16}
