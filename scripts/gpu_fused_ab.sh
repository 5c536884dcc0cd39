#!/bin/bash
# Fused update kernel A/B (REFERENCE default pipeline): update parity on the new build, then base vs new.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
BASE=${BASE:-3fs_amd/lib/libhf3fs_crc_v0.so}
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"reference": {[^}]*' gpurun_out/$name.log | grep -o 'ms_per_batch": [0-9.]*') $(tail -1 gpurun_out/$name.log | cut -c1-60)"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run t 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_dropin.py -k "update or cpp" -x -q --timeout 120 --timeout-method thread
export D3_AB=0 D3_MODES=reference
for r in 1 2 3; do
  run base$r 200 env HF3FS_CRC_LIB=$BASE python3 tests/bench_suite.py d3
  run new$r 200 python3 tests/bench_suite.py d3
done
