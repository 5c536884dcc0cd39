#!/bin/bash
# tests + C++ drop-in + seg sweep + suite + rocprof, stop at the first crash-type exit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run tests 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread
run seg 400 bash scripts/seg_sweep.sh
run suite 900 python -u bench_suite.py
bash scripts/gpu_profile.sh; echo "profile rc=$?"
