#!/bin/bash
# bench.py at N=1 (with the pinned-host H2D leg) and the 2-rank gloo rehearsal on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-1500; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bench1 300 python -u bench.py
run bench2_gloo 300 env HF3FS_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 --chunks 2048
