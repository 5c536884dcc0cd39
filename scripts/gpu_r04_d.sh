#!/bin/bash
# Round 4, call D: full GPU suite on the new defaults (hw apply body + nt stores), d3 REFERENCE
# A/B (fused kernel copy body), DELTA apply-piece sweep, then the d3 kernel trace + PMC passes.
set -eo pipefail
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/d_tests.log 2>&1
tail -1 $O/d_tests.log
for r in 1 2; do
for nt in 0 6; do
  HF3FS_CRC_APPLY_NT=$nt D3_AB=0 D3_MODES=reference SUITE_CPU=0 timeout -k 10 300 python tests/bench_suite.py d3 > $O/d3_ref_$nt.jsonl 2>/dev/null
  python -c "import json;d=json.loads(open('$O/d3_ref_$nt.jsonl').read().splitlines()[-1]);print('reference apply_nt=$nt', d['results']['reference']['ms_per_batch'])" >> $O/d3_ref_ab.log
done
done
cat $O/d3_ref_ab.log
for pm in "8 64" "4 64" "16 64" "8 128" "8 256" "8 64"; do
  set -- $pm
  HF3FS_CRC_APPLY_PIECES=$1 HF3FS_CRC_APPLY_MIN_KIB=$2 D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -k 10 300 python tests/bench_suite.py d3 > $O/d3_pieces.jsonl 2>/dev/null
  python -c "import json;d=json.loads(open('$O/d3_pieces.jsonl').read().splitlines()[-1]);print('pieces=$1 min_kib=$2', d['results']['delta']['ms_per_batch'])" >> $O/d3_pieces_sweep.log
done
cat $O/d3_pieces_sweep.log
D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_d3 -o run --output-format csv -- python3 tests/bench_suite.py d3 > $O/trace_d3.log 2>&1
D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_d3_fetch -o run --output-format csv -- python3 tests/bench_suite.py d3 > $O/pmc_d3_fetch.log 2>&1
D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_d3_write -o run --output-format csv -- python3 tests/bench_suite.py d3 > $O/pmc_d3_write.log 2>&1
AB_LIBS="f4_base f4_pf6 f4_pf8" AB_ROUNDS=6 timeout -k 10 300 python scripts/ab_f4_inproc.py > $O/f4_prefetch_ab.log 2>&1
cat $O/f4_prefetch_ab.log | tail -5
echo done
