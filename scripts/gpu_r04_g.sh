#!/bin/bash
# Round 4, call G: k_crc_run_stream (option run_stream) -- parity first, then the pre-hash matrix
# in one process, then d3 DELTA in alternating processes with run_stream 0 / 1.
set -eo pipefail
O=gpurun_out/r04/g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "run_stream or byte_runs or random_ranges or update_batch_vs or mixed_chunk or 8MiB" > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/probe_prehash_matrix.py > $O/prehash_matrix.log 2>&1
grep -h "_runs\|_rs" $O/prehash_matrix.log | cut -c1-160
for r in 1 2; do
for rs in 0 1; do
  HF3FS_CRC_RUN_STREAM=$rs D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -k 10 300 python tests/bench_suite.py d3 > $O/d3_rs_$rs.jsonl 2>/dev/null
  python -c "import json;d=json.loads(open('$O/d3_rs_$rs.jsonl').read().splitlines()[-1]);print('run_stream=$rs', d['results']['delta']['ms_per_batch'])" >> $O/d3_run_stream.log
done
done
cat $O/d3_run_stream.log
