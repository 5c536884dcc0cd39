#!/bin/bash
# HBM traffic per suite config: separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of
# tests/bench_suite.py <cfg> (no CPU legs); summarised by scripts/suite_pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp SUITE_CPU=0 D3_AB=0 D3_MODES=delta
mkdir -p gpurun_out/spmc
for cfg in ${PMC_CFGS:-d3 d4 d5 f3 f4}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== $cfg $c ($(date +%T))"
    timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/spmc/$cfg/$c -o run --output-format csv -- \
      python3 tests/bench_suite.py $cfg > gpurun_out/spmc/${cfg}_$c.log 2>&1 || exit $?
  done
done
echo suite-pmc-done
