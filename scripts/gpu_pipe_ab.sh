#!/bin/bash
# Cross-task head prefetch A/B (HF3FS_CRC_PIPE): GPU tests on the new build,
# then bench.py (d2) and the small-range configs (d5 f4) base vs new, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
BASE=${BASE:-3fs_amd/lib/libhf3fs_crc_v0.so}
CFGS=${CFGS:-d5 f4}
TESTS=${TESTS:-tests}
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/$name.log | cut -c1-360; if [ $rc -ne 0 ]; then tail -5 gpurun_out/$name.log; exit $rc; fi; }
run tests 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 180 --timeout-method thread
for r in 1 2; do
  run bbase$r 200 env HF3FS_CRC_LIB=$BASE python3 bench.py --steps 20 --warmup 3
  run bnew$r 200 python3 bench.py --steps 20 --warmup 3
  run base$r 400 env HF3FS_CRC_LIB=$BASE python3 tests/bench_suite.py $CFGS
  run new$r 400 python3 tests/bench_suite.py $CFGS
  run off$r 400 env HF3FS_CRC_PIPE=0 python3 tests/bench_suite.py $CFGS
done
