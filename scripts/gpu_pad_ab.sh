#!/bin/bash
# Lane-parallel x^(-8 pad) A/B: GPU tests on the new build, then f4 / d5 / bench, base vs new.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
BASE=${BASE:-3fs_amd/lib/libhf3fs_crc_v0.so}
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/$name.log | python3 -c '
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if "roofline" in d: print("  bench", d["value"], d["roofline"]["launch_ms_mean"], d["bit_exact"])
    elif "frames_per_s" in d: print("  f4", d["gbs"], d["ms_per_batch"], d["mismatch_set_exact"], d.get("bit_exact_sample"))
    elif "blocks_per_s" in d: print("  d5", d["gbs"], d["blocks_per_s"])
'; tail -1 gpurun_out/$name.log | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi; }
run tests 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread
for r in 1 2; do
  run base$r 400 env HF3FS_CRC_LIB=$BASE python3 tests/bench_suite.py f4 d5
  run new$r 400 python3 tests/bench_suite.py f4 d5
done
run bnew 200 python bench.py --no-cpu-baseline --h2d-chunks 0
