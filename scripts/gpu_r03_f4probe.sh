#!/bin/bash
# f4 cost split: no boundary work / no finalize vs head, one process per size class.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O; rm -f $O/f4_split.log
for cfg in "64,256,1024,4096,16384:1000000:mix" "1024:1000000:k1" "64:2000000:b64" "16384:200000:k16"; do
  IFS=: read -r sz n tag <<< "$cfg"
  echo "== f4 $tag" >> $O/f4_split.log
  AB_ROUNDS=${AB_ROUNDS:-6} AB_LIBS="${F4LIBS:-fhead fatom fnobnd fnofin}" F4_SIZES=$sz F4_N=$n timeout -k 10 180 python3 -u scripts/ab_f4_inproc.py >> $O/f4_split.log 2>&1 || { tail -5 $O/f4_split.log; exit 1; }
done
grep -v amdgpu.ids $O/f4_split.log
