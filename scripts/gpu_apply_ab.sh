#!/bin/bash
# Apply-copy A/B: update parity tests under the variant, then d3 DELTA default vs variant (alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
VAR=${VAR:-HF3FS_CRC_APPLY_SHFL=1}
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
run upd_tests_var 300 env $VAR python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_dropin.py -k "update or VerifyChecksum or cpp" -x -q --timeout 120 --timeout-method thread
export D3_AB=0 D3_MODES=delta
run d3_base1 200 python3 tests/bench_suite.py d3
run d3_var1 200 env $VAR python3 tests/bench_suite.py d3
run d3_base2 200 python3 tests/bench_suite.py d3
run d3_var2 200 env $VAR python3 tests/bench_suite.py d3
