#!/bin/bash
# Round 4, call B: byte runs past 4 GiB (parity), pre-hash matrix, d4 TLB probe (+ PMC), copy PMC calibration.
set -eo pipefail
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "byte_runs" > $O/byte_runs_tests.log 2>&1
timeout -k 10 300 python scripts/probe_prehash_matrix.py > $O/prehash_matrix.log 2>&1
timeout -k 10 300 python scripts/d4_tlb_probe.py > $O/d4_tlb.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum -d $O/pmc_d4_tlb -o run --output-format csv -- python3 scripts/d4_tlb_probe.py > $O/d4_tlb_pmc1.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_d4_fetch -o run --output-format csv -- python3 scripts/d4_tlb_probe.py > $O/d4_tlb_pmc2.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_copy_fetch -o run --output-format csv -- scratch/probe_copy 1 bodies > $O/copy_pmc1.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_copy_write -o run --output-format csv -- scratch/probe_copy 1 bodies > $O/copy_pmc2.log 2>&1

# d3 DELTA with the apply's stores / loads non-temporal (option apply_nt), alternating processes
for nt in 0 2 0 2 1 3; do
  HF3FS_CRC_APPLY_NT=$nt D3_AB=0 D3_MODES=delta SUITE_CPU=0 timeout -k 10 300 python tests/bench_suite.py d3 > $O/d3_apply_nt_$nt.jsonl 2>/dev/null
  python -c "import json;d=json.loads(open('$O/d3_apply_nt_$nt.jsonl').read().splitlines()[-1]);print('apply_nt=$nt', d['results']['delta']['ms_per_batch'])" >> $O/d3_apply_nt.log
done
echo done2
