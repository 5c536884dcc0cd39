#!/bin/bash
# bench.py A/B of two library builds, interleaved 3x (HF3FS_CRC_LIB=$BASE vs the in-tree build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
BASE=${BASE:-3fs_amd/lib/libhf3fs_crc_v0.so}
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep '^{' gpurun_out/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["launch_ms_mean"], d["bit_exact"])')"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for r in 1 2 3; do
  run base$r 200 env HF3FS_CRC_LIB=$BASE python bench.py --no-cpu-baseline --h2d-chunks 0
  run new$r 200 python bench.py --no-cpu-baseline --h2d-chunks 0
done
