"""bench.py's own multi-rank branch on the GPU box (world size 2, both ranks on
cuda:0, HF3FS_BENCH_BACKEND=gloo: collectives through host memory), launched the
way the driver launches it (torch.distributed.run, 127.0.0.1).  Checks the JSON
line: every rank's digests and the all-gathered node table equal the oracle's
golden table (bit_exact), as does the pinned-host H2D leg (streamed ring and zero-copy)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_multirank_gloo():
    env = dict(os.environ, HF3FS_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--chunks", "256", "--h2d-chunks", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints one line
    line = lines[0]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["bit_exact"] is True
    assert line["pinned_h2d"]["bit_exact"] is True  # both forms: streamed ring and zero-copy
    assert line["pinned_h2d"]["zero_copy_gbs"] > 0.0
    assert line["config"]["chunks_per_gpu"] == 256


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` typed exactly as the driver's SCALE run types it (no
    torch.distributed.run around it): bench.py starts the two ranks itself, and the
    line reports both (gloo rehearsal: both ranks on cuda:0)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HF3FS_BENCH_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--chunks", "256", "--h2d-chunks", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["collective"]["world"] == 2
    assert line["collective"]["ms_per_step"] > 0.0
    assert line["bit_exact"] is True and line["pinned_h2d"]["bit_exact"] is True


def test_bench_rccl_gpus_flag_on_one_gpu_box_exits_before_spawning():
    """The RCCL branch of `python bench.py --gpus 2` as the driver's SCALE run types it, on this
    1-GPU box: it counts the GPUs from sysfs (no HIP call, so the parent could still spawn the
    ranks), finds one, and exits non-zero before starting any rank, holding no /dev/kfd fd."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HF3FS_BENCH_BACKEND")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--chunks", "256", "--h2d-chunks", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, env=env, cwd=REPO)
    assert r.returncode != 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "--gpus 2 but 1 GPU(s) visible" in r.stderr, r.stderr[-3000:]
    assert "holds 0 /dev/kfd fd" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]  # no rank ran


def test_bench_rccl_forced_single_rank():
    """bench.py's distributed branch over RCCL ("nccl") at world size 1
    (HF3FS_BENCH_FORCE_DIST=1): the process group, the per-step digest all-gather
    through node.allgather_digests and the bit-exact check of the gathered table
    all run on the MI355X.  A single rank measures no scaling."""
    env = dict(os.environ, HF3FS_BENCH_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1", "--chunks", "512",
           "--h2d-chunks", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["collective"]["backend"] == "nccl" and line["collective"]["world"] == 1
    assert line["collective"]["ms_per_step"] >= 0.0
    assert line["bit_exact"] is True
    assert line["pinned_h2d"]["bit_exact"] is True
