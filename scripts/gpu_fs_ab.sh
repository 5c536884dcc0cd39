#!/bin/bash
# frame stream kernel: parity (both paths), then A/B of segments per wave and size classes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_aux.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/t.log)"; [ $rc -ne 0 ] && exit $rc
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u tests/bench_suite.py f4 > gpurun_out/f4s.log 2>&1; local rc=$?
  echo "$label rc=$rc $(tail -1 gpurun_out/f4s.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*\|"mismatch_set_exact": [a-z]*' | tr '\n' ' ')"
  return $rc
}
run "1GiBx3 segw1" F4_SIZES=1073741824 F4_N=3 HF3FS_CRC_FRAME_STREAM=1 HF3FS_CRC_FRAME_SEGW=1 &&
run "1GiBx3 segw2" F4_SIZES=1073741824 F4_N=3 HF3FS_CRC_FRAME_STREAM=1 &&
run "16K segw1" F4_SIZES=16384 F4_N=200000 HF3FS_CRC_FRAME_SEGW=1 &&
run "16K segw2" F4_SIZES=16384 F4_N=200000 &&
run "16K segw4" F4_SIZES=16384 F4_N=200000 HF3FS_CRC_FRAME_SEGW=4 &&
run "4K  segw2" F4_SIZES=4096 F4_N=500000 &&
run "1K  segw2" F4_SIZES=1024 F4_N=1000000 &&
run "256 segw2" F4_SIZES=256 F4_N=1000000 &&
run "64  segw2" F4_SIZES=64 F4_N=1000000 &&
run "mix segw1" F4_SIZES=64,256,1024,4096,16384 F4_N=1000000 HF3FS_CRC_FRAME_SEGW=1 &&
run "mix segw2" F4_SIZES=64,256,1024,4096,16384 F4_N=1000000 &&
run "mix segw4" F4_SIZES=64,256,1024,4096,16384 F4_N=1000000 HF3FS_CRC_FRAME_SEGW=4
