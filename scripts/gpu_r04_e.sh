#!/bin/bash
# Round 4, call E: start-aligned grid alignment A/B (pre-hash job list as byte runs, d2), in one process.
set -eo pipefail
O=gpurun_out/r04
mkdir -p $O
AB_LIBS="pre_base pre_a128 pre_a1k" AB_CASES="pre d2" timeout -k 10 400 python scripts/ab_ranges_inproc.py > $O/grid_align_ab.log 2>&1
cat $O/grid_align_ab.log
