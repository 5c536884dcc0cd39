#!/bin/bash
# f4: record path (frame_stream=0) vs stream path (frame_stream=1) per frame-size class and on
# the mix, alternating processes.  Output: gpurun_out/f4_route_ab.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/f4_route_ab.jsonl
: > $out
for rep in 1 2; do
  for sz in 64 256 1024 4096 16384 mix; do
    for fs in 0 1; do
      if [ $sz = mix ]; then envs=""; else envs="F4_SIZES=$sz F4_N=${F4_N:-1000000}"; fi
      env $envs HF3FS_CRC_FRAME_STREAM=$fs SUITE_CPU=0 timeout -k 10 240 python -u tests/bench_suite.py f4 \
        > gpurun_out/f4_route_one.log 2>&1
      rc=$?
      line=$(grep '^{' gpurun_out/f4_route_one.log)
      echo "{\"rep\": $rep, \"size\": \"$sz\", \"frame_stream\": $fs, \"line\": ${line:-null}}" >> $out
      [ $rc -le 1 ] || exit $rc
    done
  done
done
