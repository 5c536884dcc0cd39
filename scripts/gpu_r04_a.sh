#!/bin/bash
# Round 4, call A: pool-growth probe (library-free), the GPU suite, the round-start bench line.
set -eo pipefail
mkdir -p gpurun_out/r04
bash scripts/gpu_r04_pool.sh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04/gpu_tests_a.log 2>&1
tail -3 gpurun_out/r04/gpu_tests_a.log
