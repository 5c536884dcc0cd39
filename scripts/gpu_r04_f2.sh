#!/bin/bash
# Round 4, measurement pass 2: the bench suite, every leg with its CPU column.
set -eo pipefail
O=gpurun_out/r04/f2
mkdir -p $O
timeout -k 10 1000 python -u tests/bench_suite.py > $O/suite.jsonl 2> $O/suite.err
tail -c 3000 $O/suite.jsonl
