#!/bin/bash
# control: same 3 x 1 GiB receive buffer through the record path (k_crc_ranges) and the stream path; bulk d2 reference
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for m in 0 1; do
  HF3FS_CRC_FRAME_STREAM=$m F4_SIZES=1073741824 F4_N=3 timeout -k 10 200 python -u tests/bench_suite.py f4 > gpurun_out/f4s.log 2>&1; rc=$?
  echo "3GiB stream=$m rc=$rc $(tail -1 gpurun_out/f4s.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*' | tr '\n' ' ')"
  HF3FS_CRC_FRAME_STREAM=$m F4_SIZES=1073741824 F4_N=12 timeout -k 10 200 python -u tests/bench_suite.py f4 > gpurun_out/f4s.log 2>&1; rc=$?
  echo "12GiB stream=$m rc=$rc $(tail -1 gpurun_out/f4s.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --h2d-chunks 0 > gpurun_out/b.log 2>&1; echo "bench rc=$? $(tail -1 gpurun_out/b.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
