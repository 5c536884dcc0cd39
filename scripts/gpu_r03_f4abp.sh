#!/bin/bash
# The suite's f4 leg with library builds of several commits, alternating, one box; then the
# C++ drop-in test in fresh processes (plain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03; mkdir -p $O; rm -f $O/f4abp.log
for r in 1 2; do
  for lib in ${LIBS:-r3start lwonly atom}; do
    HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/$lib.so SUITE_CPU=0 timeout -k 10 200 python3 -u tests/bench_suite.py f4 > $O/f4abp_$lib.log 2>&1 || { tail -5 $O/f4abp_$lib.log; exit 1; }
    echo "$r $lib $(grep '^{' $O/f4abp_$lib.log | grep -o '"ms_per_batch": [0-9.]*\|"mismatch_set_exact": [a-z]*' | tr '\n' ' ')" >> $O/f4abp.log
  done
done
cat $O/f4abp.log
bash scripts/gpu_r03_cpprep.sh ${CPPREP:-16}
