#!/bin/bash
# Round 4, call I: one-op lookup addresses (perm-addressed step tables) and byte-table fold
# Horner -- parity (full GPU suite, smoke), then in-process A/Bs of base (HEAD before the
# change) / perm (step tables only) / permfold (both): f4 mix, 1 KiB, 16 KiB frames; d2, d5 and
# the d3 pre-hash job list; then d3 DELTA end to end in alternating processes, and bench.py.
set -eo pipefail
O=gpurun_out/r04/i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
AB_LIBS="base perm permfold pfx" timeout -k 10 300 python -u scripts/ab_f4_inproc.py > $O/f4_mix.log 2>&1
F4_SIZES=1024 F4_N=1000000 AB_LIBS="base perm permfold pfx" timeout -k 10 300 python -u scripts/ab_f4_inproc.py > $O/f4_k1.log 2>&1
F4_SIZES=16384 F4_N=200000 AB_LIBS="base perm permfold pfx" timeout -k 10 300 python -u scripts/ab_f4_inproc.py > $O/f4_k16.log 2>&1
grep -h "median" $O/f4_*.log
AB_LIBS="base perm permfold pfx" AB_CASES="d2 d5 pre" timeout -k 10 400 python -u scripts/ab_ranges_inproc.py > $O/ranges.log 2>&1
tail -12 $O/ranges.log
for r in 1 2; do
  for v in base pfx; do
    if [ $v = base ]; then export HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/base.so; else unset HF3FS_CRC_LIB; fi
    D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -k 10 300 python tests/bench_suite.py d3 > $O/d3_$v.jsonl 2>/dev/null
    python -c "import json;d=json.loads(open('$O/d3_$v.jsonl').read().splitlines()[-1]);print('$v', d['results']['delta']['ms_per_batch'], d['results']['delta']['bit_exact'])" >> $O/d3_ab.log
  done
done
unset HF3FS_CRC_LIB
cat $O/d3_ab.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cut -c1-400 $O/bench.json
