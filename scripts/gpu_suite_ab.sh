#!/bin/bash
# Library A/B on suite configs: GPU tests on the new build, then base vs new, interleaved.
#   CFGS="d4" bash scripts/gpu_suite_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
BASE=${BASE:-3fs_amd/lib/libhf3fs_crc_v0.so}
CFGS=${CFGS:-d4}
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/$name.log | cut -c1-420; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then exit $rc; fi; }
run tests 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread
for r in 1 2; do
  run base$r 400 env HF3FS_CRC_LIB=$BASE python3 tests/bench_suite.py $CFGS
  run new$r 400 python3 tests/bench_suite.py $CFGS
done
