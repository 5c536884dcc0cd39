#!/bin/bash
# A/B: the segment shift computed before the hash (xfirst) vs after the fold (base):
# d2 in one process, then the d3 pre-hash probe and the suite's d3 DELTA leg per build, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
AB_LIBS="base xfirst" AB_CASES="d2" bash scripts/gpu_r03_ab5.sh | grep "^d2" || exit 1
for r in 1 2; do
  for lib in base xfirst; do
    HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/$lib.so timeout -k 10 200 python3 -u scripts/probe_d3_prehash.py 2>&1 | grep interleaved | sed "s/^/$lib /" | cut -c1-140
    HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/$lib.so D3_MODES=delta D3_AB=0 SUITE_CPU=0 timeout -k 10 300 python3 -u tests/bench_suite.py d3 > $O/d3x.log 2>&1 || { tail -3 $O/d3x.log; exit 1; }
    echo "$lib d3 $(grep '^{' $O/d3x.log | grep -o '"delta": {[^}]*}' | grep -o '"ms_per_batch": [0-9.]*\|"bit_exact": [a-z]*' | tr '\n' ' ')"
  done
done
