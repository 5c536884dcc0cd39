#!/bin/bash
# f4 diagnostics (probe builds): in-process A/B of AB_LIBS over frame-size classes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export AB_LIBS=${AB_LIBS:-"f_head f_post"} AB_ROUNDS=${AB_ROUNDS:-6}
specs=${F4_SPECS:-16384:1000000 1048576:16000 4096:1000000 64,256,1024,4096,16384:1000000}
for spec in $specs; do
  echo "== sizes ${spec%%:*} n ${spec##*:}"
  F4_SIZES=${spec%%:*} F4_N=${spec##*:} timeout -k 10 240 python3 scripts/ab_f4_inproc.py || exit $?
done
echo f4-diag-done
