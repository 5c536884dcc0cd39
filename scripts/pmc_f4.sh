#!/bin/bash
# SQ counters of the f4 kernels per size class (one --pmc pass per config)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcf4
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"}
CFGS=${CFGS:-"16384:200000:k16 1024:1000000:k1"}
for cfg in $CFGS; do
  IFS=: read -r sz n tag <<< "$cfg"
  F4_SIZES=$sz F4_N=$n timeout -s KILL 120 rocprofv3 --pmc $CTRS -d gpurun_out/pmcf4/$tag -o run --output-format csv -- python3 -u tests/bench_suite.py f4 > gpurun_out/pmcf4/$tag.log 2>&1 || exit $?
  echo "$tag done"
done
python3 scripts/pmc_summary.py gpurun_out/pmcf4
