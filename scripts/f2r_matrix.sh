#!/bin/bash
# f2r diagnosis: gpu-reg read-result batches of 256 at 16 and 32 worker
# threads, each with a spinning, blocking and polling wait; the host CPU at 16 and 32 threads;
# then one kernel trace of the 32-thread spinning run.  -> gpurun_out/f2r_matrix.jsonl, f2r_trace/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B=tests/cpp/bench_read_batch
out=gpurun_out/f2r_matrix.jsonl
: > $out
cat /sys/fs/cgroup/cpu.stat > gpurun_out/f2r_cpu_stat_before.txt 2>/dev/null; cat /sys/fs/cgroup/cpu.max >> gpurun_out/f2r_cpu_stat_before.txt 2>/dev/null
for batch in 256 1024; do
  for th in 16 32; do
    timeout -k 10 60 $B --mode cpu --threads $th --batch $batch --seconds 2 >> $out || exit $?
    for w in spin block yield; do
      timeout -k 10 60 $B --mode gpu-reg --threads $th --batch $batch --seconds 2 --wait $w >> $out || exit $?
    done
  done
done
cat /sys/fs/cgroup/cpu.stat > gpurun_out/f2r_cpu_stat.txt 2>/dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/f2r_trace -o run --output-format csv -- \
  $B --mode gpu-reg --threads 32 --batch 256 --seconds 2 --wait spin > gpurun_out/f2r_trace.log 2>&1 || exit $?
echo f2r-matrix-done
