#!/bin/bash
# Build libhf3fs_crc.so from a git ref (or the working tree: "WT") into
# 3fs_amd/lib/ab/NAME.so for in-process A/B:  scripts/build_variant.sh NAME REF [hipcc flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; ref=$2; shift 2
d=/tmp/variant_$name; rm -rf $d; mkdir -p $d
if [ "$ref" = WT ]; then mkdir -p $d/3fs_amd && cp -r 3fs_amd/csrc $d/3fs_amd/ && cp -r include $d/; else git archive "$ref" 3fs_amd/csrc include | tar -x -C $d; fi
mkdir -p 3fs_amd/lib/ab
srcs="$(ls $d/3fs_amd/csrc/*.hip | grep -v _ab_frame) $(ls $d/3fs_amd/csrc/*.cc)"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -I $d/include "$@" -o 3fs_amd/lib/ab/$name.so $srcs
echo built 3fs_amd/lib/ab/$name.so
