#!/bin/bash
# per-kernel f4 times for library variants: LIBS="name ..." CFGS="sizes:n:tag ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
CFGS=${CFGS:-"16384:200000:k16 64,256,1024,4096,16384:1000000:mix"}
for lib in $LIBS; do
  rm -rf gpurun_out/pf4; mkdir -p gpurun_out/pf4
  for cfg in $CFGS; do
    IFS=: read -r sz n tag <<< "$cfg"
    HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/$lib.so F4_SIZES=$sz F4_N=$n timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/pf4/$tag -o run -- python3 -u tests/bench_suite.py f4 > gpurun_out/pf4/$tag.log 2>&1 || exit $?
  done
  echo "== $lib"; python3 scripts/pf4_summary.py
done
