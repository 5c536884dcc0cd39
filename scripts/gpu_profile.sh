#!/bin/bash
# rocprofv3 kernel trace + PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) of bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof; mkdir -p $OUT
ARGS=${BENCH_ARGS:-""}  # the driver's default bench command
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --h2d-chunks 0 > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --h2d-chunks 0 > $OUT/write.log 2>&1 || exit $?
echo profile-done
