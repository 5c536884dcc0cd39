#!/bin/bash
# Run one gpurun call, retrying ONLY while the pool answers "no box / slot free" (exit 3:
# nothing ran, nothing charged), every 3 minutes, at most 10 times.
#   scripts/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 10); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 180
done
exit 3
