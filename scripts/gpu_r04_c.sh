#!/bin/bash
# Round 4, call C: d3 DELTA apply-body / nt-store A/B (alternating processes), parity of the hw body,
# then the d3 kernel trace of the winner and its PMC passes.
set -eo pipefail
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
HF3FS_CRC_APPLY_NT=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "update or byte_runs or random_ranges or d5" > $O/hw_body_tests.log 2>&1
tail -1 $O/hw_body_tests.log
for r in 1 2; do
for nt in 0 2 4 6; do
  HF3FS_CRC_APPLY_NT=$nt D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -k 10 300 python tests/bench_suite.py d3 > $O/d3_c_$nt.jsonl 2>/dev/null
  python -c "import json;d=json.loads(open('$O/d3_c_$nt.jsonl').read().splitlines()[-1]);print('apply_nt=$nt', d['results']['delta']['ms_per_batch'])" >> $O/d3_apply_body.log
done
done
cat $O/d3_apply_body.log
# d4 geometry: task size sweep on the 64 GiB batch (separate processes, alternating)
for r in 1 2; do
for seg in 4096 16384 8192 65536; do
  HF3FS_CRC_SEG_KIB=$seg timeout -k 10 200 python scripts/d4_probe.py >> $O/d4_seg_sweep.log 2>/dev/null
done
done
cat $O/d4_seg_sweep.log
