#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcd5
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"}
for k in 4 64; do
  D5_KIB=$k timeout -s KILL 90 rocprofv3 --pmc $CTRS -d gpurun_out/pmcd5/k$k -o run --output-format csv -- python3 -u scripts/d5_size_probe.py > gpurun_out/pmcd5/k$k.log 2>&1 || exit $?
  tail -1 gpurun_out/pmcd5/k$k.log
done
python3 scripts/pmc_summary.py gpurun_out/pmcd5 | grep -E "==|k_crc_ranges"
