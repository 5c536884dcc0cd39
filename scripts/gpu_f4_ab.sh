#!/bin/bash
# f4 A/B over library variants: LIBS="name ..." (3fs_amd/lib/ab/NAME.so), CFGS="sizes:n:tag ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/f4ab
CFGS=${CFGS:-"16384:200000:k16 1024:1000000:k1 64,256,1024,4096,16384:1000000:mix"}
for cfg in $CFGS; do
  IFS=: read -r sz n tag <<< "$cfg"
  for lib in $LIBS; do
    HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/$lib.so F4_SIZES=$sz F4_N=$n timeout -k 10 120 python3 -u tests/bench_suite.py f4 > gpurun_out/f4ab/$tag.$lib.log 2>&1; rc=$?
    echo "$tag $lib rc=$rc $(grep '^{' gpurun_out/f4ab/$tag.$lib.log | grep -o '"gbs": [0-9.]*\|"ms_per_batch": [0-9.]*\|"mismatch_set_exact": [a-z]*\|"bit_exact_sample": [a-z]*' | tr '\n' ' ')"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
