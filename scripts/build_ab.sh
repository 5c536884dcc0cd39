#!/bin/bash
# Build A/B variants of libhf3fs_crc.so that differ only in frame_kernels.hip:
#   scripts/build_ab.sh NAME FRAME_SOURCE [extra hipcc flags...]
# -> 3fs_amd/lib/ab/NAME.so (load with HF3FS_CRC_LIB=...).  Other sources are
# compiled once into /tmp/abobj.
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
C=3fs_amd/csrc; O=/tmp/abobj; mkdir -p $O 3fs_amd/lib/ab
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I include"
for s in crc_kernels update_kernels digest_kernels hf3fs_crc_api coalescer aux_kernels; do
  fresh=1
  for dep in $C/$s.hip $C/*.h include/hf3fs_crc.h; do [ $O/$s.o -nt $dep ] || fresh=0; done
  [ $fresh = 1 ] || hipcc $F -c $C/$s.hip -o $O/$s.o
done
fresh=1
for dep in $C/host_codec.cc $C/*.h include/hf3fs_crc.h; do [ $O/host_codec.o -nt $dep ] || fresh=0; done
[ $fresh = 1 ] || hipcc $F -c $C/host_codec.cc -o $O/host_codec.o
cp "$src" $C/_ab_frame_$name.hip  # one file per variant: builds may run in parallel
hipcc $F "$@" -c $C/_ab_frame_$name.hip -o $O/frame_$name.o; rm -f $C/_ab_frame_$name.hip
hipcc --offload-arch=gfx950 -shared -fPIC -o 3fs_amd/lib/ab/$name.so $O/{crc_kernels,update_kernels,digest_kernels,hf3fs_crc_api,coalescer,aux_kernels,host_codec}.o $O/frame_$name.o
echo built 3fs_amd/lib/ab/$name.so
