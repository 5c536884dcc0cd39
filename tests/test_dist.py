"""Multi-rank path on CPU (gloo, world_size 2): chain-id sharding and the digest
all-gather of 3fs_amd/node.py.  On the GPU node the same code runs over RCCL;
here each rank's shard is hashed by the oracle as a stand-in for the device."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SEED = 0x3F5C3C00


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_chunks, num_chains, length, q, equal_shards=False):
    import importlib
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "oracle"))
    import oracle
    node = importlib.import_module("3fs_amd.node")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = node.shard_chunk_ids(n_chunks, rank, world, num_chains)
        num_chains = num_chains or n_chunks
        crcs = np.array([oracle.crc32c_raw(oracle.fill_synth(length, SEED, int(i))) for i in ids], dtype=np.uint32)
        all_ids, all_crcs = node.allgather_digests(torch.from_numpy(ids), torch.from_numpy(crcs.astype(np.int64)),
                                                   world, shard_size=ids.size if equal_shards else None)
        q.put((rank, ids.tolist(), all_ids.tolist(), all_crcs.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_chunks,num_chains,equal", [(16, 2, False), (13, 3, False), (1, 2, False),
                                                       (16, None, False), (9, 5, False), (16, None, True)])
def test_chain_sharded_allgather(orc, n_chunks, num_chains, equal):
    """equal: bench.py's form -- equal shards, shard_size given, no count exchange."""
    world, length = 2, 10000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_chunks, num_chains, length, q, equal))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [orc.crc32c_raw(orc.fill_synth(length, SEED, i)) for i in range(n_chunks)]
    num_chains = num_chains or n_chunks
    import importlib
    node = importlib.import_module("3fs_amd.node")
    owned = []
    for rank, ids, all_ids, all_crcs in results:
        assert all_ids == list(range(n_chunks))
        assert all_crcs == expect
        lo, hi = node.chain_range(rank, world, num_chains)
        assert all(lo <= i % num_chains < hi for i in ids)
        assert list(node.owner_of_chain([i % num_chains for i in ids], world, num_chains)) == [rank] * len(ids)
        owned += ids
    assert sorted(owned) == list(range(n_chunks))  # every chunk hashed exactly once


def test_allgather_shard_size_must_match():
    """a shard_size that is not this rank's id count is an error, not padding rows in the table."""
    import importlib
    node = importlib.import_module("3fs_amd.node")
    with pytest.raises(ValueError, match="shard_size"):
        node.allgather_digests(torch.arange(3), torch.zeros(3, dtype=torch.int64), 2, backend="gloo", shard_size=4)


def test_bench_gpus_launch_decision():
    """bench.py --gpus N: with no WORLD_SIZE and N > 1 it starts N ranks through a child
    torch.distributed.run (127.0.0.1); a --gpus that disagrees with WORLD_SIZE is an error."""
    import importlib
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    bench = importlib.import_module("bench")
    assert bench.check_world(1, {}) == "run"
    assert bench.check_world(8, {}) == "launch"
    assert bench.check_world(2, {"WORLD_SIZE": "2"}) == "run"
    assert "WORLD_SIZE=4" in bench.check_world(8, {"WORLD_SIZE": "4"})
    assert "WORLD_SIZE=1" in bench.check_world(2, {"WORLD_SIZE": "1"})
    assert "must be" in bench.check_world(0, {})
    cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "5"], 4, 12345)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4" and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"] and cmd[-5].endswith("bench.py")


def test_bench_gpus_mismatch_exits_nonzero():
    """The mismatch check runs before anything touches a GPU, so it is exercised on the CPU."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=repo)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_visible_gpus_from_sysfs(tmp_path):
    """bench.visible_gpus counts GPUs without a HIP call: KFD topology nodes with SIMDs whose
    render node opens, capped by the *_VISIBLE_DEVICES lists (a fake topology here)."""
    import importlib
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    bench = importlib.import_module("bench")
    topo, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    spec = {0: (0, None), 1: (256, 128), 2: (256, 129), 3: (256, 130)}  # node: (simd_count, render minor)
    for node, (simd, minor) in spec.items():
        d = topo / str(node)
        d.mkdir(parents=True)
        text = f"cpu_cores_count 8\nsimd_count {simd}\n" + (f"drm_render_minor {minor}\n" if minor else "")
        (d / "properties").write_text(text)
    for minor in (128, 129):  # node 3's render node is not there (a device cgroup hides it)
        (dri / f"renderD{minor}").write_text("")
    assert bench.visible_gpus({}, str(topo), str(dri)) == 2
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "0"}, str(topo), str(dri)) == 1
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": "0,1,2"}, str(topo), str(dri)) == 2
    assert bench.visible_gpus({}, str(tmp_path / "none"), str(dri)) == 0
    assert bench.kfd_fds() == 0


def test_bench_rccl_launch_without_gpus_exits_nonzero():
    """`bench.py --gpus 2` over RCCL on a host with fewer GPUs stops before it spawns, and
    says how many it saw, without touching the GPU (this container has none)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HF3FS_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=repo)
    assert r.returncode != 0 and "--gpus 2 but 0 GPU(s) visible" in r.stderr, r.stderr
    assert "holds 0 /dev/kfd fd" in r.stderr
