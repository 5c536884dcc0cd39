#!/bin/bash
# f4 (tests/bench_suite.py f4): kernel trace + one SQ counter pass (8 SQ counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trf4 -o run --output-format csv -- \
  python3 tests/bench_suite.py f4 > gpurun_out/trf4.log 2>&1 || exit $?
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
timeout -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/pmcf4 -o run --output-format csv -- \
  python3 tests/bench_suite.py f4 > gpurun_out/pmcf4.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmcf4 > gpurun_out/pmcf4_summary.txt
echo f4-profile-done
