#!/bin/bash
# Service-mode diagnosis (C++ per-IO bench, then the opt-in pytest cases) and a
# d3 per-kernel profile.  Each step is time-limited; crash-type exits stop the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 3 ] && [ $rc -ne 4 ]; then exit $rc; fi; }
B=./tests/cpp/bench_coalescer
run svc_t1 60 $B --mode service-hbm --threads 1 --seconds 0.5 --arena-mib 256 --service-wgs 8
run svc_t32 60 $B --mode service-hbm --threads 32 --seconds 1 --arena-mib 256 --service-wgs 32
run coal_t32 60 $B --mode coalesced-hbm --threads 32 --seconds 1 --arena-mib 256
run svc_tests 240 python -u -m pytest tests/test_coalescer.py -v --timeout 60 --timeout-method thread
mkdir -p gpurun_out/p3d
export D3_MODES=delta
run prof_d3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p3d -o run --output-format csv -- python3 tests/bench_suite.py d3
echo done
