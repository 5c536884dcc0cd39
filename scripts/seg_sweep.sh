#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for seg in 256 1024 2048 4096; do
  HF3FS_CRC_SEG_KIB=$seg timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/seg_$seg.log 2>&1 || exit $?
  echo "seg=$seg $(python -c "import json,sys; d=json.loads(open('gpurun_out/seg_$seg.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['launch_ms_mean'])")"
done
