#!/bin/bash
# Round-3 probes: f4 fold cost (conflict-free / no-multiply fold variants vs head, in one
# process), the d5 gather-only probe, and the d4 streamed-H2D probe + trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O
for cfg in "64,256,1024,4096,16384:1000000:mix" "1024:1000000:k1" "16384:200000:k16" "64:2000000:b64"; do
  IFS=: read -r sz n tag <<< "$cfg"
  echo "== f4 $tag" >> $O/f4_foldprobe.log
  AB_LIBS="head lw cf nomul" F4_SIZES=$sz F4_N=$n timeout -k 10 180 python3 -u scripts/ab_f4_inproc.py >> $O/f4_foldprobe.log 2>&1 || { tail -5 $O/f4_foldprobe.log; exit 1; }
done
cat $O/f4_foldprobe.log
timeout -k 10 300 ./build/probe_gather 5 > $O/gather_probe.log 2>&1 || { cat $O/gather_probe.log; exit 1; }
cat $O/gather_probe.log
bash scripts/gpu_r03_h2d.sh
