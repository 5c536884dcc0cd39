#!/bin/bash
# round 6: copy probe (library-shaped one-shot legs) + d3 PMC traffic, one-shot vs ticketed apply
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_copy_ceiling.hip -o /tmp/pcc || exit 1
timeout -k 10 200 /tmp/pcc 7 ragged > gpurun_out/r06_copy_ceiling6.log 2>&1 || exit $?
for g in 0 -1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    HF3FS_CRC_APPLY_GRID=$g D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -s KILL 150 rocprofv3 --pmc $c \
      -d gpurun_out/pmc_d3_g${g}_$c -o run --output-format csv -- python3 tests/bench_suite.py d3 \
      > gpurun_out/pmc_d3_g${g}_$c.log 2>&1 || exit $?
  done
done
