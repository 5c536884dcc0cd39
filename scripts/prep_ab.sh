#!/bin/bash
# d3 prep geometry A/B (probe): kernel trace of the d3 suite config per library build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp D3_AB=0 D3_MODES=delta SUITE_CPU=0
mkdir -p gpurun_out
for r in 1 2; do
  for lib in ${AB_LIBS:-p256 p128 p64}; do
    export HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/$lib.so
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prep_${lib}_$r -o run --output-format csv -- \
      python3 tests/bench_suite.py d3 > gpurun_out/prep_${lib}_$r.log 2>&1 || exit $?
    python3 scripts/kstats.py gpurun_out/prep_${lib}_$r | grep -E "update_prep|apply_one|List" | sed "s/^/$lib r$r /"
    grep '^{' gpurun_out/prep_${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib r$r', 'd3 delta ms', d['results']['delta']['ms_per_batch'])"
    rm -rf gpurun_out/prep_${lib}_$r
  done
done
echo prep-ab-done
