#!/bin/bash
# d3 DELTA pre-hash segment size A/B (separate processes, one box) + this box's d2 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03; mkdir -p $O
export D3_MODES=delta D3_AB=0 SUITE_CPU=0
timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --h2d-chunks 0 > $O/seg_bench.log 2>&1 || exit $?
tail -1 $O/seg_bench.log | cut -c1-300
for rep in 1 2; do
for seg in 256 512 1024 128; do
  HF3FS_CRC_SEG_KIB=$seg timeout -k 10 120 python3 tests/bench_suite.py d3 > $O/seg_$seg.log 2>&1 || exit $?
  echo "seg=$seg $(tail -1 $O/seg_$seg.log | grep -o '"delta": {[^}]*}')"
done
done
