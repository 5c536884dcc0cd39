#!/bin/bash
# Round 4, call C: parity of the new paths (range_stream kernel, hw apply body), then A/Bs in
# alternating processes: d5 range_stream 0/1, d3 DELTA apply body / nt stores, d4 task size.
set -eo pipefail
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
HF3FS_CRC_APPLY_NT=6 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "update or byte_runs or random_ranges or d5 or range_stream or many_small" > $O/c_tests.log 2>&1
tail -1 $O/c_tests.log
for r in 1 2; do
for rs in 0 1; do
  HF3FS_CRC_RANGE_STREAM=$rs SUITE_CPU=0 timeout -k 10 300 python tests/bench_suite.py d5 > $O/d5_rs_$rs.jsonl 2>/dev/null
  python -c "import json;d=json.loads(open('$O/d5_rs_$rs.jsonl').read().splitlines()[-1]);print('range_stream=$rs', d.get('ms_total'), d.get('gbs'), d.get('mismatch_set_exact'), d.get('bit_exact_sample'))" >> $O/d5_range_stream.log
done
done
cat $O/d5_range_stream.log
for r in 1 2; do
for nt in 0 2 4 6; do
  HF3FS_CRC_APPLY_NT=$nt D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -k 10 300 python tests/bench_suite.py d3 > $O/d3_c_$nt.jsonl 2>/dev/null
  python -c "import json;d=json.loads(open('$O/d3_c_$nt.jsonl').read().splitlines()[-1]);print('apply_nt=$nt', d['results']['delta']['ms_per_batch'])" >> $O/d3_apply_body.log
done
done
cat $O/d3_apply_body.log
for r in 1 2; do
for seg in 4096 16384 8192 65536; do
  HF3FS_CRC_SEG_KIB=$seg timeout -k 10 200 python scripts/d4_probe.py >> $O/d4_seg_sweep.log 2>/dev/null
done
done
cat $O/d4_seg_sweep.log
