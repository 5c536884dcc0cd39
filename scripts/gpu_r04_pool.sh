#!/bin/bash
# Round 4: library-free probe of freshly grown / re-mapped pool memory, then the
# round-start bench line.
set -eo pipefail
mkdir -p gpurun_out/r04
B=scratch/probe_pool_growth
for m in trim grow reuse malloc; do
  for st in null own; do
    timeout -k 10 120 $B 400 $m $st memcpy >> gpurun_out/r04/pool_probe.log
  done
done
for k in $(seq 1 24); do timeout -k 10 60 $B 2 grow null memcpy >> gpurun_out/r04/pool_probe_fresh.log; done
for k in $(seq 1 8); do timeout -k 10 60 $B 1 trim null memcpy >> gpurun_out/r04/pool_probe_fresh.log; done
timeout -k 10 300 python bench.py > gpurun_out/r04/bench_start.json 2> gpurun_out/r04/bench_start.err
cat gpurun_out/r04/pool_probe.log
