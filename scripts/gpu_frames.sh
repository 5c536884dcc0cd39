#!/bin/bash
# f4 stream path: frame parity (both paths), then f4 per size class and the mix, stream vs record.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_aux.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/t.log)"; [ $rc -ne 0 ] && exit $rc
for cfg in "64 1000000" "256 1000000" "1024 1000000" "4096 500000" "16384 200000" "64,256,1024,4096,16384 1000000"; do
  set -- $cfg
  for m in 1 0; do
    HF3FS_CRC_FRAME_STREAM=$m F4_SIZES=$1 F4_N=$2 timeout -k 10 200 python -u tests/bench_suite.py f4 > gpurun_out/f4s.log 2>&1; rc=$?
    echo "f4 sizes=$1 stream=$m rc=$rc $(tail -1 gpurun_out/f4s.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*\|"mismatch_set_exact": [a-z]*\|"bit_exact_sample": [a-z]*' | tr '\n' ' ')"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
