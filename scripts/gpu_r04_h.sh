#!/bin/bash
# Round 4, call H: SQ counters of k_frame_stream (f4) per frame-size class, two --pmc passes each.
set -eo pipefail
O=gpurun_out/r04/h
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT"
run() {  # tag sizes n
  for p in 1 2; do
    if [ $p = 1 ]; then C=$P1; else C=$P2; fi
    F4_SIZES=$2 F4_N=$3 timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$1_p$p -o run --output-format csv -- python3 -u tests/bench_suite.py f4 > $O/$1_p$p.log 2>&1
  done
}
run k16 16384 200000
run k1 1024 1000000
run mix "" ""
python3 scripts/pmc_summary.py $O > $O/summary.txt
cat $O/summary.txt
