#!/bin/bash
# Apply row alignment A/B: parity under 4 KiB rows, then d3 DELTA with ALIGN 0 / 1 KiB / 4 KiB interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_batch": [0-9.]*' gpurun_out/$name.log | head -1) $(tail -1 gpurun_out/$name.log | cut -c1-80)"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run t4 300 env HF3FS_CRC_APPLY_ALIGN=4 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_dropin.py -k "update or cpp" -x -q --timeout 120 --timeout-method thread
export D3_AB=0 D3_MODES=delta
for r in 1 2; do
  for a in 0 1 4; do run d3_a${a}_r$r 200 env HF3FS_CRC_APPLY_ALIGN=$a python3 tests/bench_suite.py d3; done
done
