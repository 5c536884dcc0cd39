#!/bin/bash
# Named GPU steps for one gpurun call, each under its own time limit, stopping at the
# first crash-type exit (anything but 0 / 1):
#   bash scripts/gpu_steps.sh tests smoke bench profile suite soak ...
# Logs go to gpurun_out/<step>.log.  Knobs: SUITE_CASES, SOAK_SECONDS, AB_LIBS, AB_CASES,
# LIBTEST (a 3fs_amd/lib/ab/NAME.so to run the -m gpu suite against).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for step in "$@"; do
  case $step in
    tests) run tests 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread ;;
    libtests) HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/$LIBTEST.so run libtests_$LIBTEST 600 \
                python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -k "not cpp and not bench_" ;;
    smoke) run smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python -u bench.py ;;
    profile) echo "== profile ($(date +%T))"; bash scripts/gpu_profile.sh; rc=$?; echo "profile rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    suite) run suite 900 python -u tests/bench_suite.py ${SUITE_CASES:-} ;;
    soak) run soak $(( ${SOAK_SECONDS:-240} + 120 )) python -u tests/soak.py ${SOAK_SECONDS:-240} ;;
    profd3) mkdir -p gpurun_out/p3; D3_AB=0 D3_MODES=delta SUITE_CPU=0 run profd3 300 rocprofv3 --kernel-trace --stats \
              -d gpurun_out/p3 -o run --output-format csv -- python3 tests/bench_suite.py d3 ;;
    proff4) mkdir -p gpurun_out/p4; run proff4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p4 -o run \
              --output-format csv -- python3 tests/bench_suite.py f4 && \
            run pmcf4 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES \
              SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d gpurun_out/p4pmc -o run --output-format csv -- \
              python3 tests/bench_suite.py f4 ;;
    ab) run ab 600 python -u scripts/ab_ranges_inproc.py ;;
    abf4) run abf4 300 python -u scripts/ab_f4_inproc.py ;;
    abd3) for r in $(seq 1 ${AB_ROUNDS:-2}); do for lib in $AB_LIBS; do
            HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/$lib.so D3_AB=0 D3_MODES=delta SUITE_CPU=0 \
              run abd3_${lib}_$r 300 python -u tests/bench_suite.py d3
          done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo all-steps-done
