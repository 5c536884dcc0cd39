#!/bin/bash
# Kernel trace of the f4 suite leg per frame-size class (which kernel holds the time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
for cfg in "64,256,1024,4096,16384:1000000:mix" "1024:1000000:k1" "64:2000000:b64"; do
  IFS=: read -r sz n tag <<< "$cfg"
  SUITE_CPU=0 F4_SIZES=$sz F4_N=$n timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/f4trace_$tag -o run --output-format csv -- python3 -u tests/bench_suite.py f4 > $O/f4trace_$tag.log 2>&1 || { tail -5 $O/f4trace_$tag.log; exit 1; }
  echo "== $tag $(grep '^{' $O/f4trace_$tag.log | grep -o '"ms_per_batch": [0-9.]*')"
  python3 scripts/kstats.py $O/f4trace_$tag 12 || true
done
