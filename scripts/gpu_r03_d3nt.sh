#!/bin/bash
# d3 pre-hash probe and the suite's d3 DELTA leg with non-temporal (default) vs cached loads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
for nt in 1 0 1 0; do
  HF3FS_CRC_NT=$nt timeout -k 10 200 python3 -u scripts/probe_d3_prehash.py 2>&1 | grep probe | sed "s/^/nt=$nt /"
  HF3FS_CRC_NT=$nt D3_MODES=delta D3_AB=0 SUITE_CPU=0 timeout -k 10 300 python3 -u tests/bench_suite.py d3 > $O/d3nt.log 2>&1 || { tail -3 $O/d3nt.log; exit 1; }
  echo "nt=$nt d3 $(grep '^{' $O/d3nt.log | grep -o '"delta": {[^}]*}' | grep -o '"ms_per_batch": [0-9.]*')"
done
