#!/usr/bin/env python3
"""bench.py -- CRC32C chunk-integrity throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "Bulk write path"): 4096 chunks x 4 MiB
(16 GiB) resident in HBM per GPU; one step = ChecksumInfo::create(CRC32C) over
the whole batch in one launch (hf3fs_crc_create_strided) and, for N > 1, the
RCCL all-gather of the per-chunk digest table (the path's only exchange step;
chunks are sharded by chain id -- contiguous chain-table ranges per GPU -- so
per-GPU work is fixed: weak scaling).

Prints ONE JSON line (rank 0).  `value` = bytes hashed by all ranks / max step
time.  `roofline.achieved` = algorithmic bytes per launch / the launch's mean
duration from HIP events on the launch stream.  `cpu_baseline` = the oracle's
folly::crc32c restatements (SSE4.2 3-way and carry-less folding; the faster is `value`)
timed on this host over config 0's sample (rank 0, N=1 only).  `pinned_h2d` = the PCIe-inclusive rate of config 3's shape
(64 MiB chunks streamed from pinned host memory; `zero_copy_gbs` the same bytes read in place from
registered pageable memory), aggregated over all ranks.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--chunks C] [--chunk-mib M]
  torchrun --nproc-per-node N bench.py --gpus N ...
`python bench.py --gpus N` (N > 1, no WORLD_SIZE) starts the N ranks itself as a child
torch.distributed.run; a --gpus that disagrees with WORLD_SIZE exits non-zero.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
SEED = 0x3F5C3C00
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "CRC32C GB/s per GPU & per node (4 MiB chunks) + % HBM peak, bit-exact"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chunks", type=int, default=4096)
    ap.add_argument("--chunk-mib", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = every core this job may use: affinity and cgroup quota)")
    ap.add_argument("--h2d-chunks", type=int, default=16,
                    help="64 MiB chunks per GPU in the pinned-host H2D leg (0 = skip)")
    return ap.parse_args()


def host_cpus():
    """Cores this job may run on: the affinity mask, capped by a cgroup v2 CPU quota
    (a GPU box's share is a quota; nproc / os.cpu_count() show the whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return {"usable": usable, "nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "model": model}


def cpu_baseline(threads, L=None, hf=None, dev=None):
    """BASELINE configs[0]: 1024 x 512 KiB synthetic chunks, ChecksumInfo::create
    semantics (1 MiB slices, Common.h:146-177) on every core this job may use and on one
    core, in two CPU forms of folly::crc32c (Common.h:158): the SSE4.2 3-way crc32
    instruction stream, and carry-less-multiply folding (AVX-512 VPCLMULQDQ, else
    PCLMULQDQ), the algorithm class folly's large-buffer x86 dispatch uses in current
    releases (the folly commit the reference pins is unrecorded).  `value`
    is the faster all-core form.  Each figure is the median of >= 7 passes.  The same 1024
    chunks are then hashed on the device (one hf3fs_crc_create_strided launch, outside any
    timed region) and compared bit for bit with every oracle digest of both forms
    (north_star: bit-exact against the folly::crc32c path on identical synthetic chunks)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test/baseline infrastructure only

    n, length = 1024, 512 << 10
    data = np.empty((n, length), dtype=np.uint8)
    for i in range(n):
        data[i] = oracle.fill_synth(length, SEED, i)
    cpus = host_cpus()
    threads = max(1, threads or cpus["usable"])
    forms = {"sse42": 0, "clmul": 2}
    res = {}
    for name, kind in forms.items():
        for t in sorted({1, threads}):
            oracle.create_batch(data[:64], threads=t, kind=kind)  # warm
            runs = []
            t_end = time.perf_counter() + (2.5 if t == 1 else 1.5)
            while time.perf_counter() < t_end or len(runs) < 7:
                t0 = time.perf_counter()
                oracle.create_batch(data, threads=t, kind=kind)
                runs.append(time.perf_counter() - t0)
            res[name, t] = (n * length / 1e9) / float(np.median(runs))
    digests = {name: np.asarray(oracle.create_batch(data, threads=threads, kind=kind), dtype=np.uint32)
               for name, kind in forms.items()}
    cpu_digests = digests["sse42"]
    best = max(forms, key=lambda f: res[f, threads])
    lib = oracle.lib()
    clmul_form = "VPCLMULQDQ" if lib.orc_have_vpclmul() else "PCLMULQDQ" if lib.orc_have_clmul() else "SSE4.2 fallback"
    out = {"value": round(res[best, threads], 2), "unit": "GB/s", "cores": threads, "kind": "port",
           "form": best,
           "sse42_gbs": {"single_core": round(res["sse42", 1], 2), "all_cores": round(res["sse42", threads], 2)},
           "clmul_gbs": {"single_core": round(res["clmul", 1], 2), "all_cores": round(res["clmul", threads], 2),
                         "isa": clmul_form},
           "sample": f"1024 x 512 KiB synthetic chunks (512 MiB), median of >= 7 passes per form and core count; "
                     f"oracle/crc_oracle.c: SSE4.2 3-way crc32 and {clmul_form} folding (folly::crc32c "
                     f"restatements); value = the faster ({best}) on {threads} cores",
           "single_core_gbs": round(res[best, 1], 2), "forms_bit_exact": bool(np.array_equal(*digests.values())),
           "host": cpus}
    if L is not None:
        d = torch.from_numpy(data).to(dev)
        g = torch.zeros(n, dtype=torch.int32, device=dev)
        L.create_strided(hf.CRC32C, d, length, length, n, g, stream=torch.cuda.current_stream(dev))
        torch.cuda.synchronize(dev)
        gpu_digests = g.cpu().numpy().view(np.uint32)
        out["cpu_gpu_bit_exact"] = bool(np.array_equal(gpu_digests, cpu_digests))
        out["cpu_gpu_check"] = ("the same 1024 x 512 KiB chunks hashed on the device (hf3fs_crc_create_strided) vs "
                                "all 1024 oracle digests of this leg (ChecksumInfo::create, Common.h:146-177)")
        del d
    return out


def h2d_leg(L, hf, dev, rank, n_chunks, steps=2, chunk=64 << 20, slots=4):
    """BASELINE configs[3] shape, PCIe-inclusive: n_chunks x 64 MiB per GPU in
    pinned host memory, streamed H2D through a `slots`-deep device ring on as
    many streams, each piece hashed on its stream right after its copy lands; then
    the zero-copy form (pageable memory, hf3fs_crc_host_register, one launch).
    Reported beside `value`, never as it (the HBM-resident rate is `value`).
    Chunks are ids [rank n, (rank + 1) n) of the 64 MiB synthetic stream, checked
    against the oracle's golden table (tests/golden/bulk_64MiB_digests.bin)."""
    s = torch.cuda.current_stream(dev)
    dsrc = torch.empty(n_chunks * chunk, dtype=torch.uint8, device=dev)
    L.fill_synth(dsrc, chunk, chunk, n_chunks, SEED, rank * n_chunks, stream=s)
    host = torch.empty(n_chunks * chunk, dtype=torch.uint8, pin_memory=True)
    host.copy_(dsrc)
    del dsrc
    ref = None
    gdir = os.path.join(REPO, "tests", "golden")
    g = np.fromfile(os.path.join(gdir, "bulk_64MiB_digests.bin"), dtype="<u4")
    if (rank + 1) * n_chunks <= g.size:
        ref = torch.from_numpy(g[rank * n_chunks:(rank + 1) * n_chunks].view(np.int32).copy()).to(dev)
    ring = [torch.empty(chunk, dtype=torch.uint8, device=dev) for _ in range(slots)]
    streams = [torch.cuda.Stream(dev) for _ in range(slots)]
    hout = torch.zeros(n_chunks, dtype=torch.int32, device=dev)

    def one_pass():
        for i in range(n_chunks):
            k = i % slots
            with torch.cuda.stream(streams[k]):
                ring[k].copy_(host[i * chunk:(i + 1) * chunk], non_blocking=True)
                L.create_strided(hf.CRC32C, ring[k], chunk, chunk, 1, hout[i:i + 1], stream=streams[k])

    one_pass()
    torch.cuda.synchronize(dev)
    ok = None if ref is None else torch.equal(hout, ref)
    hout.zero_()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_pass()
    torch.cuda.synchronize(dev)
    sec = time.perf_counter() - t0
    if ref is not None:
        ok = ok and torch.equal(hout, ref)
    # zero-copy: the same bytes in pageable host memory registered through the library
    # (hf3fs_crc_host_register, as 3FS registers its RDMA BufferPool); one create_strided
    # launch reads the mapped pages over PCIe, no device copy
    pageable = torch.empty(n_chunks * chunk, dtype=torch.uint8)
    pageable.copy_(host)
    del host
    dptr = L.host_register(pageable.data_ptr(), n_chunks * chunk)
    try:
        s0 = torch.cuda.current_stream(dev)
        zout = torch.zeros(n_chunks, dtype=torch.int32, device=dev)
        L.create_strided(hf.CRC32C, dptr, chunk, chunk, n_chunks, zout, stream=s0)
        torch.cuda.synchronize(dev)
        if ref is not None:
            ok = ok and torch.equal(zout, ref)
        zout.zero_()
        t0 = time.perf_counter()
        for _ in range(steps):
            L.create_strided(hf.CRC32C, dptr, chunk, chunk, n_chunks, zout, stream=s0)
        torch.cuda.synchronize(dev)
        zsec = time.perf_counter() - t0
        if ref is not None:
            ok = ok and torch.equal(zout, ref)
    finally:
        L.host_unregister(pageable.data_ptr())
    return sec, zsec, n_chunks * chunk * steps, ok


def launcher_cmd(argv, n, port):
    """The child command `bench.py --gpus N` (N > 1, no WORLD_SIZE) runs: one rank per GPU
    through torch.distributed.run on 127.0.0.1, the same bench.py arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def check_world(gpus, env):
    """Returns "launch" (start N ranks as a child), "run" (this process is the rank) or an
    error string.  A --gpus that disagrees with the launcher's WORLD_SIZE fails loudly:
    the line's n_gpus is always the number of ranks that were timed."""
    if gpus < 1:
        return f"--gpus {gpus}: must be >= 1"
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else "run"
    if int(ws) != gpus:
        return f"WORLD_SIZE={ws} but --gpus {gpus}: launch {gpus} ranks or pass --gpus {ws}"
    return "run"


def kfd_fds():
    """Open /dev/kfd descriptors of this process (0 before anything initialises HIP)."""
    n = 0
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                n += os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd"
            except OSError:
                pass
    except OSError:
        pass
    return n


def visible_gpus(env=None, sysfs="/sys/class/kfd/kfd/topology/nodes", dev_dir="/dev/dri"):
    """GPUs this process may use, counted WITHOUT any HIP call (the launcher decides before
    anything touches the GPU; exec'ing after HIP initialised is forbidden on this pool):
    KFD topology nodes with SIMDs (GPU agents) whose DRM render node this process can
    open -- a container's device cgroup hides the rest -- capped by the
    HIP/ROCR/CUDA_VISIBLE_DEVICES lists.  No amdsmi and no hipGetDeviceCount fallback."""
    env = os.environ if env is None else env
    n = 0
    try:
        nodes = os.listdir(sysfs)
    except OSError:
        nodes = []
    for node in nodes:
        props = {}
        try:
            with open(os.path.join(sysfs, node, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
        except OSError:
            continue
        if int(props.get("simd_count", "0") or 0) <= 0:
            continue  # a CPU agent
        minor = props.get("drm_render_minor")
        if minor is None:
            continue
        try:
            fd = os.open(os.path.join(dev_dir, f"renderD{int(minor)}"), os.O_RDWR | os.O_CLOEXEC)
            os.close(fd)
        except (OSError, ValueError):
            continue
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(args):
    """`python bench.py --gpus N` with N > 1: start N ranks as a CHILD process before this
    process touches the GPU, and exit with its return code.  RCCL needs a GPU per rank,
    counted by visible_gpus() from sysfs (no HIP call); the gloo rehearsal
    (HF3FS_BENCH_BACKEND=gloo) shares the visible GPUs."""
    import socket
    import subprocess
    if os.environ.get("HF3FS_BENCH_BACKEND", "nccl") == "nccl":
        have = visible_gpus()
        if have < args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but {have} GPU(s) visible "
                     f"(KFD topology + render nodes; this process holds {kfd_fds()} /dev/kfd fd)")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return subprocess.call(launcher_cmd(sys.argv[1:], args.gpus, port), env=env)


def main():
    args = parse()
    what = check_world(args.gpus, os.environ)
    if what == "launch":
        sys.exit(launch_ranks(args))
    if what != "run":
        sys.exit("bench.py: " + what)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL ("nccl") over xGMI in production; HF3FS_BENCH_BACKEND=gloo is a
    # rehearsal mode for the multi-rank logic on a 1-GPU box (ranks share cuda:0,
    # collectives go through host memory).
    backend = os.environ.get("HF3FS_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local_rank = local_rank % max(1, torch.cuda.device_count())
    # HF3FS_BENCH_FORCE_DIST=1: the distributed branch (process group + digest all-gather) at
    # world size 1 too, so a 1-GPU box runs RCCL once (no scaling claim comes from it).
    use_dist = world > 1 or os.environ.get("HF3FS_BENCH_FORCE_DIST") == "1"
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local_rank)

    def allreduce(t, op):
        if not use_dist:
            return
        if backend == "nccl":
            dist.all_reduce(t, op=op)
        else:
            c = t.cpu()
            dist.all_reduce(c, op=op)
            t.copy_(c)
    hf = importlib.import_module("3fs_amd")
    node = importlib.import_module("3fs_amd.node")
    L = hf._lib
    L.load()

    n, length = args.chunks, args.chunk_mib << 20
    total_local = n * length
    buf = torch.empty(total_local, dtype=torch.uint8, device=dev)
    # chain-id sharding (3fs_amd/node.py): every chunk its own chain, GPU r owns the
    # contiguous chain-table range [r n, (r + 1) n) of the node's n * world chunks
    ids = node.shard_chunk_ids(n * world, rank, world)
    assert ids.size == n and int(ids[-1]) - int(ids[0]) == n - 1
    first_id = int(ids[0])
    stream = torch.cuda.current_stream(dev)
    L.fill_synth(buf, length, length, n, SEED, first_id, stream=stream)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    ids_dev = torch.from_numpy(ids).to(dev)
    gathered = [None]  # the node's digest table (node.allgather_digests: ids, crcs), ordered by chunk id

    def gather():  # the path's one exchange step: the chain-sharded digest tables, RCCL all-gather
        if use_dist:
            gathered[0] = node.allgather_digests(ids_dev, out, world, backend=backend, shard_size=n)

    for _ in range(args.warmup):
        L.create_strided(hf.CRC32C, buf, length, length, n, out, stream=stream)
        gather()
    torch.cuda.synchronize(dev)

    # timed region: barrier + sync on both sides, exactly K steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    # the exchange step's own time: from the hash's end event to an event recorded after the
    # all-gather + cat + argsort on the same stream (torch orders RCCL's stream before it)
    evg = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)] if use_dist else []
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        L.create_strided(hf.CRC32C, buf, length, length, n, out, stream=stream)
        ev[k][1].record(stream)
        gather()
        if use_dist:
            evg[k].record(stream)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    coll_ms = float(np.mean([ev[k][1].elapsed_time(evg[k]) for k in range(args.steps)])) if use_dist else 0.0

    t = torch.tensor([elapsed, launch_ms, coll_ms], dtype=torch.float64, device=dev)
    allreduce(t, dist.ReduceOp.MAX)
    elapsed, launch_ms_max, coll_ms_max = float(t[0]), float(t[1]), float(t[2])

    # bit-exactness: the whole digest table (every rank's, and the all-gathered
    # node table, compared where it was gathered) against the oracle's
    # full-size golden table, committed data (tests/golden/make_bulk_golden.py);
    # no oracle code runs on this leg.
    gdir = os.path.join(REPO, "tests", "golden")
    golden = None
    gname = f"bulk_{args.chunk_mib}MiB_digests"
    if os.path.exists(os.path.join(gdir, gname + ".json")):
        with open(os.path.join(gdir, gname + ".json")) as f:
            gmeta = json.load(f)
        if length == gmeta["chunk_bytes"] and world * n <= gmeta["chunks"]:
            g = np.fromfile(os.path.join(gdir, gname + ".bin"), dtype="<u4")[:world * n]
            golden = torch.from_numpy(g.view(np.int32).copy()).to(dev)
    bit_exact = None  # no golden table for a chunk size / count without one
    if golden is not None:
        bit_exact = bool(torch.equal(out, golden[first_id:first_id + n]))
        if use_dist:
            g_ids, g_crcs = gathered[0]
            bit_exact = (bit_exact and bool(torch.equal(g_ids, torch.arange(world * n, device=dev)))
                         and bool(torch.equal(g_crcs, golden.to(torch.int64) & 0xFFFFFFFF)))
    if use_dist:  # codes ordered so that MAX keeps a failure: 0 unchecked, 1 ok, 2 mismatch
        flag = torch.tensor([0 if bit_exact is None else (1 if bit_exact else 2)], device=dev)
        allreduce(flag, dist.ReduceOp.MAX)
        bit_exact = None if int(flag.item()) == 0 else int(flag.item()) == 1

    total_bytes = total_local * world
    value = total_bytes * args.steps / elapsed / 1e9
    achieved = total_local / (launch_ms / 1e3) / 1e9
    traffic, traffic_src = None, None
    pmc = os.path.join(REPO, "profiles", "pmc_bulk_4096x4MiB.json")
    if os.path.exists(pmc) and n == 4096 and length == 4 << 20:
        with open(pmc) as f:
            pm = json.load(f)
        traffic = pm.get("hbm_bytes_per_launch")
        traffic_src = (f"{os.path.relpath(pmc, REPO)} ({pm.get('round')}): FETCH_SIZE x2 + WRITE_SIZE per launch from "
                       f"separate rocprofv3 --pmc passes of this command, NOT counted in this run")

    h2d = None
    if args.h2d_chunks > 0:
        if use_dist:
            dist.barrier()
        sec, zsec, nbytes, ok = h2d_leg(L, hf, dev, rank, args.h2d_chunks)
        # verdict codes ordered so that MAX over ranks keeps a failure: 0 unchecked, 1 ok, 2 mismatch
        t = torch.tensor([sec, zsec, 0.0 if ok is None else (1.0 if ok else 2.0)], dtype=torch.float64, device=dev)
        allreduce(t, dist.ReduceOp.MAX)
        h2d = {"value": round(nbytes * world / float(t[0]) / 1e9, 2), "unit": "GB/s",
               "per_gpu_gbs": round(nbytes / float(t[0]) / 1e9, 2),
               "zero_copy_gbs": round(nbytes * world / float(t[1]) / 1e9, 2),
               "bit_exact": None if float(t[2]) == 0.0 else float(t[2]) == 1.0,
               "bit_exact_check": "every digest of both forms vs tests/golden/bulk_64MiB_digests.bin (oracle)",
               "sample": f"{args.h2d_chunks} x 64 MiB per GPU in host memory (BASELINE configs[3] shape), 2 passes "
                         f"per form; value: pinned memory, 4-slot device ring on 4 streams, copy + hash per piece; "
                         f"zero_copy_gbs: pageable memory registered by hf3fs_crc_host_register, one launch reads "
                         f"the mapped pages; max time over ranks; PCIe-inclusive, reported beside value, never as it"}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64, SURVEY.md §8d), HBM-resident",
            "config": {"workload": f"bulk write path: {n} x {args.chunk_mib} MiB chunks CRC32C per GPU "
                                   f"(BASELINE configs[1]), hf3fs_crc_create_strided",
                       "chunks_per_gpu": n, "chunk_bytes": length,
                       "parallelism": f"chain-sharded x{world}" + (" + RCCL digest all-gather" if use_dist else "")},
            "per_gpu_gbs": round(value / world, 2),
            "pct_hbm_peak": round(100.0 * achieved / HBM_PEAK_GBS, 2),
            "bit_exact": bit_exact,
            "bit_exact_check": f"every digest of every rank + the all-gathered table (on the device) vs "
                               f"tests/golden/{gname}.bin (oracle/crc_oracle.c, pinned by the reference KATs)",
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_crc_ranges<CRC32C, whole-buffer tasks, NT loads>",
                         "launch_ms_mean": round(launch_ms, 4), "launch_ms_max_over_ranks": round(launch_ms_max, 4),
                         "algorithmic_bytes_per_launch": total_local},
            "pinned_h2d": h2d,
            "cpu_baseline": None,
            "collective": ({"backend": backend, "world": world, "op": "all_gather of (chunk id, crc) digests",
                            "path": "3fs_amd/node.py allgather_digests", "per_step": True,
                            "ms_per_step": round(coll_ms, 4), "ms_per_step_max_over_ranks": round(coll_ms_max, 4),
                            "timed": "HIP events on the launch stream: hash end -> after all_gather + cat + "
                                     "argsort (rank 0's mean; max over ranks beside it)"}
                           if use_dist else None),
        }
        if not args.no_cpu_baseline and world == 1:  # the CPU leg runs on rank 0 at N=1 only
            del buf
            torch.cuda.empty_cache()
            line["cpu_baseline"] = cpu_baseline(args.cpu_threads, L, hf, dev)
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
