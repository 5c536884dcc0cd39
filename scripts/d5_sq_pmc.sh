#!/bin/bash
# SQ counters of the d5 verify kernel for all-4 KiB and all-64 KiB KV blocks (same bytes,
# scripts/d5_size_probe.py), one rocprofv3 --pmc pass per block size (8 SQ counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
for k in 4 64; do
  D5_KIB=$k timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmcd5/k$k -o run --output-format csv -- \
    python3 scripts/d5_size_probe.py > gpurun_out/pmcd5_k$k.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py gpurun_out/pmcd5 > gpurun_out/pmcd5_summary.txt
echo d5-pmc-done
