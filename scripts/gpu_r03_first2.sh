#!/bin/bash
# The first DELTA update of a process after REFERENCE updates (the C++ drop-in test's failing
# call), in fresh processes, with variants that isolate the cause.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03; mkdir -p $O; rm -f $O/first2.log
for opt in ref200 ref200,sync ref200,trim ref200,grow ref5 ref200,warm; do
  for i in $(seq 1 ${REPS:-12}); do
    timeout -k 5 60 ./build/probe_first_call 1 $opt >> $O/first2.log 2>&1 || { echo "rc=$? at $opt $i"; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
c = collections.defaultdict(lambda: [0, 0, 0])
for line in open("gpurun_out/r03/first2.log"):
    if line.startswith("{"):
        r = json.loads(line)
        k = r["opt"]
        c[k][0] += 1
        c[k][1] += r["first_status"] != 0
        c[k][2] += r["retry_status"] != 0
for k, v in c.items():
    print(f"{k:14s} runs {v[0]:3d} first_bad {v[1]:3d} retry_bad {v[2]:3d}")
PY
