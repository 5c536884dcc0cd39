#!/bin/bash
# fused DELTA A/B: piece size x copy lag on the d3 workload (default pipeline only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for cfg in ${CFGS:-"512 64" "512 256" "512 1024" "256 256" "256 1024" "1024 256"}; do
  set -- $cfg
  HF3FS_CRC_DELTA_PIECE_KIB=$1 HF3FS_CRC_DELTA_LAG=$2 D3_MODES=delta D3_AB=0 timeout -k 10 200 python -u tests/bench_suite.py d3 > gpurun_out/d3ab.log 2>&1; rc=$?
  echo "piece=$1 lag=$2 rc=$rc $(tail -1 gpurun_out/d3ab.log | grep -o '"ms_per_batch": [0-9.]*' | head -1)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
