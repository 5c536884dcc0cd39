#!/bin/bash
# Library A/B: all GPU tests on the new build, then bench.py / d5 / d3 with the
# baseline build (HF3FS_CRC_LIB=$BASE) and the new one, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
BASE=${BASE:-3fs_amd/lib/libhf3fs_crc_v0.so}
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-700; if [ $rc -ne 0 ]; then exit $rc; fi; }
run tests 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread
export D3_AB=0 D3_MODES=delta
for r in 1 2; do
  run bench_base$r 200 env HF3FS_CRC_LIB=$BASE python bench.py --no-cpu-baseline --h2d-chunks 0
  run bench_new$r 200 python bench.py --no-cpu-baseline --h2d-chunks 0
  run d5_base$r 300 env HF3FS_CRC_LIB=$BASE python3 tests/bench_suite.py d5
  run d5_new$r 300 python3 tests/bench_suite.py d5
  run d3_base$r 200 env HF3FS_CRC_LIB=$BASE python3 tests/bench_suite.py d3
  run d3_new$r 200 python3 tests/bench_suite.py d3
done
