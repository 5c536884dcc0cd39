#!/usr/bin/env python3
"""tests/bench_suite.py -- the secondary BASELINE.json configurations (one JSON line each).

  d3  ragged partial-chunk updates: 4096 resident 4 MiB chunks, one write per
      chunk per batch (len U[64 KiB, 1 MiB], byte-granular offsets, 10% appends,
      5% past-the-end writes with a zero-filled gap), hf3fs_crc_update_batch in
      DELTA and REFERENCE modes; parity = chunk checksum vs oracle after the run.
  d4  node scale, 64 MiB chunks on this GPU: HBM-resident, pinned-host streamed
      H2D (hipMemcpyAsync ring on 2 streams overlapped with hashing) and
      zero-copy (kernel reads mapped pinned host memory).
  d5  KVCache read-verify: blocks of {4,8,16,32,64} KiB at 4 KiB-aligned offsets
      of an HBM arena, verified in 1M-block batches replayed from hipGraphs;
      0.01% of expected values corrupted -> the mismatch set must be exact.
  a2  combine_batch: 16M element-wise ChecksumInfo::combine of lengths up to 64 MiB,
      every result vs the oracle's C combine (also the CPU baseline).
  f1  file digest: the admin checksum fold over 50k files x 64 chunk read checksums
      (5% short reads zero-filled, 1% missing), --fill-zero and strict modes;
      parity = the oracle's C fold on the first 4k files, also the CPU baseline.
  f2  per-IO read path: 32 threads hashing one {4..64} KiB block per call
      (AioReadJob::setResult shape) through the coalescer (HBM, registered host
      memory, host copy), one launch per IO without it, and the CPU oracle;
      driven by tests/cpp/bench_coalescer (C++ threads).
  f3  scrub: 4096 stored 4 MiB chunks re-hashed against persisted checksums
      (half raw ChunkMetadata values, half finalized ChunkMeta values), 0.1%
      corrupted -> the mismatch set must be exact.
  f4  serde frames: 1M framed messages of {64..16384} B in one HBM receive
      buffer, calcSerde verify; the host framing walk timed separately.
The primary metric (configs[1]) is bench.py.  `python tests/bench_suite.py [d3 d4 d5 a2 f1 f2 f2r f3 f4]`; it lives under tests/ because its parity checks call the oracle (test infrastructure).
"""
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # tests/ -> repo root
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402  (checker + CPU baseline only)

hf = importlib.import_module("3fs_amd")
L = hf._lib
SEED = 0x3F5C3C00
PEAK = 8000.0
DEV = torch.device("cuda:0")


def emit(d):
    print(json.dumps(d), flush=True)


def cpu_cores():
    """Every core this job may use (affinity, cgroup quota): bench.host_cpus."""
    import bench
    return bench.host_cpus()


def cpu_d3(sample=512, chunk=4 << 20):
    """CPU (N cores) baseline of d3: the reference's ChunkReplica::update per IO --
    payload verify, gap fill + write, prefix and suffix re-hashed from the chunk
    (ChunkReplica.cc:193-207, 281-292, 356-389) -- on `sample` IOs of the d3
    distribution, oracle/crc_oracle.c over every usable core."""
    cpus = cpu_cores()
    rng = np.random.default_rng(3)
    chunks = np.empty((sample, chunk), dtype=np.uint8)
    for i in range(sample):
        chunks[i] = oracle.fill_synth(chunk, SEED, i)
    sizes = rng.integers(2 << 20, chunk + 1, sample).astype(np.uint32)
    cks = np.array([oracle.crc32c_raw(chunks[i, :sizes[i]]) for i in range(sample)], dtype=np.uint32)
    lens = rng.integers(64 << 10, (1 << 20) + 1, sample).astype(np.uint32)
    offs = np.array([rng.integers(0, chunk - ln + 1) for ln in lens], dtype=np.uint32)
    r = rng.random(sample)
    app = (r < 0.10) & (sizes + lens <= chunk)
    offs[app] = sizes[app]
    gap = (r >= 0.10) & (r < 0.15) & (sizes.astype(np.int64) + lens + 4096 <= chunk)
    offs[gap] = sizes[gap] + rng.integers(1, 4097, gap.sum()).astype(np.uint32)
    payload = np.empty((sample, 1 << 20), dtype=np.uint8)
    for i in range(sample):
        payload[i] = oracle.fill_synth(1 << 20, SEED ^ 0xABCD, i)
    wcks = np.array([oracle.crc32c_raw(payload[i, :lens[i]]) for i in range(sample)], dtype=np.uint32)
    t0 = time.perf_counter()
    st = oracle.replica_update_batch(chunks, payload, sizes, cks, offs, lens, wcks, threads=cpus["usable"])
    sec = time.perf_counter() - t0
    assert not st.any()
    pay = int(lens.astype(np.int64).sum())
    return {"label": f"CPU ({cpus['usable']} cores)", "ios_per_s": round(sample / sec), "payload_gbs":
            round(pay / sec / 1e9, 2), "cores": cpus["usable"], "kind": "port", "host": cpus,
            "sample": f"{sample} updates of the d3 distribution on 4 MiB chunks, reference algorithm "
                      f"(verify + write + prefix/suffix re-hash), oracle/crc_oracle.c SSE4.2"}


def cpu_create(n, length, label_cfg):
    """CPU (N cores) ChecksumInfo::create over n synthetic chunks of `length` bytes."""
    cpus = cpu_cores()
    data = np.empty((n, length), dtype=np.uint8)
    for i in range(n):
        data[i] = oracle.fill_synth(length, SEED, i)
    oracle.create_batch(data[:1], threads=1)
    t0 = time.perf_counter()
    oracle.create_batch(data, threads=cpus["usable"])
    sec = time.perf_counter() - t0
    return {"label": f"CPU ({cpus['usable']} cores)", "gbs": round(n * length / sec / 1e9, 2), "cores": cpus["usable"],
            "kind": "port", "host": cpus, "sample": f"{n} x {length >> 20} MiB synthetic chunks ({label_cfg}), "
                                                    f"oracle/crc_oracle.c SSE4.2 3-way"}


def cpu_d5(n=1_000_000, arena=2 << 30):
    """CPU (N cores) baseline of d5: verify n KV blocks of {4..64} KiB at 4 KiB-aligned
    offsets of a host arena against expected CRCs (StorageClientImpl.cc:1720-1737)."""
    cpus = cpu_cores()
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, arena, dtype=np.uint8)
    lens = (rng.choice([4, 8, 16, 32, 64], n) * 1024).astype(np.uint32)
    offs = (rng.integers(0, (arena - 65536) // 4096, n) * 4096).astype(np.uint64)
    exp = np.zeros(n, dtype=np.uint32)
    _, _ = oracle.verify_blocks(a, offs[:1000], lens[:1000], exp[:1000], threads=1)
    t0 = time.perf_counter()
    bad, _ = oracle.verify_blocks(a, offs, lens, exp, threads=cpus["usable"])
    sec = time.perf_counter() - t0
    logical = int(lens.astype(np.int64).sum())
    return {"label": f"CPU ({cpus['usable']} cores)", "blocks_per_s": round(n / sec), "gbs": round(logical / sec / 1e9, 2),
            "cores": cpus["usable"], "kind": "port", "host": cpus,
            "sample": f"{n} blocks of {{4..64}} KiB in a {arena >> 30} GiB host arena, oracle/crc_oracle.c SSE4.2"}


_WARM = {}


def warm_gpu(seconds=0.1):
    """Keep the GPU busy for `seconds` (hashing a 1 GiB scratch buffer) right before every timed
    region: the suite reports steady-state rates.  After host-side setup the first tens of
    milliseconds of device work run slower (scripts/diag_f4.py: the suite's f4 batch 1.015 ms as
    the first measurement of a process, 0.826-0.837 ms after it, profiles/r05_f4_warmup_diag.log;
    d4's 64 GiB hash 6.43 TB/s right after its fill, 6.95 in a warm process,
    profiles/r05_d4_geometry_ab.log; bench.py's trace settles after ~10 launches)."""
    if "buf" not in _WARM:
        _WARM["buf"] = torch.zeros(1 << 30, dtype=torch.uint8, device=DEV)
        _WARM["out"] = torch.zeros(1024, dtype=torch.int32, device=DEV)
    s = torch.cuda.current_stream()
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        for _ in range(20):
            L.create_strided(hf.CRC32C, _WARM["buf"], 1 << 20, 1 << 20, 1024, _WARM["out"], stream=s)
        torch.cuda.synchronize()


def timed(fn, steps, warmup, stream):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, a.elapsed_time(b) / 1e3 / steps


# ------------------------------------------------------------------------------------------
def d3_ragged(n=4096, chunk=4 << 20, batches=8):
    """Both update modes; each also with the three-pass pipeline
    (library option update_pipeline) on the same seeded plan, for the A/B."""
    s = torch.cuda.current_stream()
    res = {}
    modes = [(hf.MODE_DELTA, "delta"), (hf.MODE_REFERENCE, "reference")]
    if os.environ.get("D3_MODES"):
        modes = [m for m in modes if m[1] in os.environ["D3_MODES"].split(",")]
    variants = [("", None)] + ([] if os.environ.get("D3_AB") == "0" else [("_unfused", "unfused"), ("_fused", "fused")])
    for mode, name in modes:
        for suffix, force in variants:  # "" = the library's default pipeline for the mode
            with L.option("update_pipeline", force or "mode"):
                res[name + suffix] = _d3_run(n, chunk, batches, mode, name, s)
    # A/B of library options in this process, DELTA: D3_OPTS="tag:opt=v,opt=v;tag2:..." (each
    # variant twice, alternating)
    spec = [v for v in os.environ.get("D3_OPTS", "").split(";") if v]
    for rep in range(2 if spec else 0):
        for v in spec:
            tag, _, kv = v.partition(":")
            pairs = [p.split("=") for p in kv.split(",") if p]
            saved = [(k, L.get_option(k)) for k, _ in pairs]
            for k, val in pairs:
                L.set_option(k, val)
            try:
                res[f"delta_{tag}_{rep}"] = _d3_run(n, chunk, batches, hf.MODE_DELTA, "delta", s)
            finally:
                for k, val in saved:
                    L.set_option(k, val)
    cpu = cpu_d3() if os.environ.get("SUITE_CPU", "1") == "1" else None
    emit({"config": "d3 ragged partial-chunk updates (BASELINE configs[2])", "chunks": n, "chunk_bytes": chunk,
          "batches": batches, "write_len": "U[64 KiB, 1 MiB]", "dtype": "u8", "results": res, "cpu": cpu,
          "note": "moved = verify read + old read (delta) or prefix/suffix re-read (reference) + copy read + write; "
                  "min = the bytes an update must touch once: payload read + old read (delta) + write"})


def _d3_run(n, chunk, batches, mode, name, s):
    rng = np.random.default_rng(3)
    if True:
        chunks = torch.empty(n * chunk, dtype=torch.uint8, device=DEV)
        L.fill_synth(chunks, chunk, chunk, n, SEED, 0, stream=s)
        sizes = rng.integers(2 << 20, chunk + 1, n).astype(np.int64)
        cks = torch.zeros(n, dtype=torch.int32, device=DEV)
        A = torch.tensor(((chunks.data_ptr() + np.arange(n) * chunk).astype(np.uint64)).view(np.int64), device=DEV)
        Ls = torch.tensor(sizes, device=DEV)
        L.create_batch(hf.CRC32C, A, Ls, cks, n, chunk, stream=s)
        payload = torch.empty(n * (1 << 20), dtype=torch.uint8, device=DEV)
        # plan all batches on the host (sizes evolve deterministically: every write verifies)
        plans = []
        for b in range(batches):
            lens = rng.integers(64 << 10, (1 << 20) + 1, n)
            offs = np.array([rng.integers(0, chunk - l + 1) for l in lens])
            r = rng.random(n)
            app = (r < 0.10) & (sizes + lens <= chunk)
            offs[app] = sizes[app]
            gap = (r >= 0.10) & (r < 0.15) & (sizes + lens + 4096 <= chunk)
            offs[gap] = sizes[gap] + rng.integers(1, 4097, gap.sum())
            plans.append((offs.copy(), lens.copy(), sizes.copy()))
            sizes = np.maximum(sizes, offs + lens)
        # payload checksums (payload bytes fixed: synth per chunk id)
        L.fill_synth(payload, 1 << 20, 1 << 20, n, SEED ^ 0xABCD, 0, stream=s)
        P = torch.tensor(((payload.data_ptr() + np.arange(n) * (1 << 20)).astype(np.uint64)).view(np.int64),
                         device=DEV)
        ios_dev = []
        for offs, lens, sz in plans:
            pl = torch.tensor(lens.astype(np.int64), device=DEV)
            pck = torch.zeros(n, dtype=torch.int32, device=DEV)
            L.create_batch(hf.CRC32C, P, pl, pck, n, 1 << 20, stream=s)
            torch.cuda.synchronize()
            arr = (hf.UpdateIO * n)()
            pck_h = pck.cpu().numpy().astype(np.uint32)
            for i in range(n):
                u = arr[i]
                u.chunk = chunks.data_ptr() + i * chunk
                u.payload = payload.data_ptr() + i * (1 << 20)
                u.offset, u.length, u.chunk_size = int(offs[i]), int(lens[i]), int(sz[i])
                u.update_type = hf.UPDATE_WRITE
                u.chunk_checksum_type = hf.CRC32C
                u.write_checksum_type, u.write_checksum = hf.CRC32C, int(pck_h[i])
            ios_dev.append(torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(DEV))
        # chain the checksums: each batch's chunk_checksum = previous batch's out (device-side copy)
        stride = ctypes.sizeof(hf.UpdateIO)

        def chain_in(ios, prev_ck):
            v = ios.view(torch.int32).view(n, stride // 4)
            v[:, 8] = prev_ck  # chunk_checksum (byte offset 32)

        # Each batch's stored checksums are the previous batch's results, as a caller's chunk
        # metadata holds them.  An untimed pass over a snapshot of the chunks finds them, so the
        # timed loop is update calls only (until round 5 a device copy per batch chained them
        # inside the timed region, ~8 us per batch).
        pristine = [t.clone() for t in ios_dev]
        snap = chunks.clone()
        ck = cks.clone()
        given = []
        for ios in ios_dev:
            chain_in(ios, ck)
            given.append(ck.clone())
            L.update_batch(hf.CRC32C, ios, n, chunk, mode=mode, stream=s)
            ck = ios.view(torch.int32).view(n, stride // 4)[:, 11]  # out_checksum (byte 44)
        chunks.copy_(snap)
        del snap
        for ios, rec, g in zip(ios_dev, pristine, given):
            ios.copy_(rec)
            chain_in(ios, g)
        del pristine, given
        torch.cuda.synchronize()
        warm_gpu()  # (the plans above are seconds of host work)
        # batch 0 is the warmup (first-use kernel loads, stream-ordered pool growth): untimed
        L.update_batch(hf.CRC32C, ios_dev[0], n, chunk, mode=mode, stream=s)
        plans = plans[1:]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(s)
        for ios in ios_dev[1:]:
            L.update_batch(hf.CRC32C, ios, n, chunk, mode=mode, stream=s)
        ev1.record(s)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        dev_s = ev0.elapsed_time(ev1) / 1e3
        last = (hf.UpdateIO * n).from_buffer_copy(ios_dev[-1].cpu().numpy().tobytes())
        ok = all(last[i].status == 0 for i in range(n))
        for i in rng.choice(n, 4, replace=False):
            h = chunks[int(i) * chunk:int(i) * chunk + last[int(i)].out_size].cpu().numpy()
            ok = ok and oracle.crc32c_raw(h) == last[int(i)].out_checksum
        payload_bytes = sum(int(p[1].sum()) for p in plans)
        old_bytes = sum(int(np.clip(np.minimum(p[0] + p[1], p[2]) - p[0], 0, None).sum()) for p in plans)
        chunk_bytes_after = sum(int(np.maximum(p[2], p[0] + p[1]).sum()) for p in plans)
        if name == "delta":  # verify read + old read + copy read + write
            moved = 2 * payload_bytes + old_bytes + payload_bytes
            minimal = payload_bytes + old_bytes + payload_bytes
        else:  # verify read + copy read + write + prefix/suffix re-read
            moved = 2 * payload_bytes + payload_bytes + (chunk_bytes_after - payload_bytes)
            minimal = payload_bytes + payload_bytes + (chunk_bytes_after - payload_bytes)
        out = {"payload_gbs": round(payload_bytes / dev_s / 1e9, 1), "updates_per_s": round(n * len(plans) / dev_s),
               "moved_gbs": round(moved / dev_s / 1e9, 1), "frac_hbm": round(moved / dev_s / 1e9 / PEAK, 3),
               "min_gbs": round(minimal / dev_s / 1e9, 1), "frac_hbm_min": round(minimal / dev_s / 1e9 / PEAK, 3),
               "ms_per_batch": round(dev_s / len(plans) * 1e3, 3), "wall_ms_per_batch": round(wall / len(plans) * 1e3, 3),
               "bit_exact": bool(ok)}
        del chunks, payload, ios_dev
        torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------------------------------------
def d4_node(n_chunks=1024, chunk=64 << 20, host_chunks=32, steps=3):
    s = torch.cuda.current_stream()
    out = torch.zeros(n_chunks, dtype=torch.int32, device=DEV)
    buf = torch.empty(n_chunks * chunk, dtype=torch.uint8, device=DEV)  # 64 GiB resident
    L.fill_synth(buf, chunk, chunk, n_chunks, SEED, 0, stream=s)
    fn = lambda: L.create_strided(hf.CRC32C, buf, chunk, chunk, n_chunks, out, stream=s)  # noqa: E731
    warm_gpu()
    wall, dev_s = timed(fn, steps, 1, s)
    hbm = n_chunks * chunk / dev_s / 1e9
    # every digest vs the oracle's golden table of the 64 MiB stream (tests/golden/make_bulk_golden.py)
    golden = np.fromfile(os.path.join(REPO, "tests", "golden", "bulk_64MiB_digests.bin"), dtype="<u4")
    ok = bool(np.array_equal(out.cpu().numpy().astype(np.uint32), golden[:n_chunks]))
    ref = torch.from_numpy(golden[:host_chunks].view(np.int32).copy()).to(DEV)
    del buf
    torch.cuda.empty_cache()

    # pinned host source (host_chunks x 64 MiB), streamed H2D through a 2-slot ring on 2 streams
    host = torch.empty(host_chunks * chunk, dtype=torch.uint8, pin_memory=True)
    dsrc = torch.empty(host_chunks * chunk, dtype=torch.uint8, device=DEV)
    L.fill_synth(dsrc, chunk, chunk, host_chunks, SEED, 0, stream=s)
    torch.cuda.synchronize()
    host.copy_(dsrc.cpu())
    del dsrc
    ring = [torch.empty(chunk, dtype=torch.uint8, device=DEV) for _ in range(4)]
    streams = [torch.cuda.Stream() for _ in range(4)]
    hout = torch.zeros(host_chunks, dtype=torch.int32, device=DEV)

    def h2d_pass():
        for i in range(host_chunks):
            k = i % 4
            with torch.cuda.stream(streams[k]):
                ring[k].copy_(host[i * chunk:(i + 1) * chunk], non_blocking=True)
                L.create_strided(hf.CRC32C, ring[k], chunk, chunk, 1, hout[i:i + 1], stream=streams[k])

    h2d_pass()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        h2d_pass()
    torch.cuda.synchronize()
    h2d = host_chunks * chunk * steps / (time.perf_counter() - t0) / 1e9
    ok = ok and torch.equal(hout, ref)

    # zero-copy: the kernel reads the mapped pinned pages directly over PCIe
    zc = torch.zeros(host_chunks, dtype=torch.int32, device=DEV)
    hipmod = ctypes.CDLL("libamdhip64.so")
    dptr = ctypes.c_void_p()
    rc = hipmod.hipHostGetDevicePointer(ctypes.byref(dptr), ctypes.c_void_p(host.data_ptr()), 0)
    zc_gbs = None
    if rc == 0:
        fz = lambda: L.create_strided(hf.CRC32C, dptr.value, chunk, chunk, host_chunks, zc, stream=s)  # noqa: E731
        wall_z, dev_z = timed(fz, steps, 1, s)
        zc_gbs = round(host_chunks * chunk / dev_z / 1e9, 1)
        ok = ok and torch.equal(zc, ref)
    emit({"config": "d4 node scale, 64 MiB chunks, this GPU (BASELINE configs[3])", "chunks": n_chunks,
          "chunk_bytes": chunk, "hbm_resident_gbs": round(hbm, 1), "frac_hbm": round(hbm / PEAK, 4),
          "pinned_h2d_streamed_gbs": round(h2d, 1), "zero_copy_pinned_gbs": zc_gbs,
          "h2d_note": "PCIe Gen5 x16 bound (63 GB/s spec)", "bit_exact": bool(ok),
          "bit_exact_check": "all 1024 digests (HBM) and every host-path digest vs tests/golden/bulk_64MiB_digests.bin",
          "cpu": cpu_create(16, chunk, "d4 shape") if os.environ.get("SUITE_CPU", "1") == "1" else None,
          "multi_gpu": "bench.py --gpus N shards chunks by chain id; digests all-gathered over RCCL"})


# ------------------------------------------------------------------------------------------
def d5_kv(n_total=10_000_000, batch=1_000_000, arena_gib=32, corrupt_frac=1e-4):
    rng = np.random.default_rng(5)
    s = torch.cuda.current_stream()
    arena_bytes = arena_gib << 30
    arena = torch.empty(arena_bytes, dtype=torch.uint8, device=DEV)
    L.fill_synth(arena, 1 << 30, 1 << 30, arena_gib, SEED, 0, stream=s)
    nb = n_total // batch
    lens_all = (rng.choice([4, 8, 16, 32, 64], n_total) * 1024).astype(np.uint32)
    offs_all = (rng.integers(0, (arena_bytes - 65536) // 4096, n_total) * 4096).astype(np.uint64)
    O = torch.tensor(offs_all.view(np.int64), device=DEV)
    Ls = torch.tensor(lens_all.view(np.int32), device=DEV)
    exp = torch.zeros(n_total, dtype=torch.int32, device=DEV)
    addrs = torch.tensor((offs_all + np.uint64(arena.data_ptr())).view(np.int64), device=DEV)
    L.create_batch(hf.CRC32C, addrs, Ls.to(torch.int64), exp, n_total, 65536, stream=s)  # expected (list path)
    torch.cuda.synchronize()
    del addrs
    bad = np.sort(rng.choice(n_total, int(n_total * corrupt_frac), replace=False))
    flip = torch.tensor((1 << rng.integers(0, 31, bad.size)).astype(np.int32), device=DEV)
    bidx = torch.tensor(bad, device=DEV)
    exp[bidx] = exp[bidx] ^ flip
    mism = torch.zeros(n_total, dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(nb, dtype=torch.int32, device=DEV)
    comp = torch.zeros(n_total, dtype=torch.int32, device=DEV)

    def run_batch(b, stream):
        sl = slice(b * batch, (b + 1) * batch)
        L.verify_blocks(hf.CRC32C, arena, O[sl], Ls[sl], exp[sl], mism[sl], cnt[b:b + 1], batch, 65536,
                        computed=comp[sl], stream=stream)

    # capture one hipGraph per batch (descriptor slices are fixed), replay all
    graphs = []
    cs = torch.cuda.Stream()
    for b in range(nb):
        run_batch(b, cs)  # warm the path on the capture stream
    torch.cuda.synchronize()
    for b in range(nb):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cs):
            run_batch(b, cs)
        graphs.append(g)
    torch.cuda.synchronize()
    for g in graphs:
        g.replay()
    torch.cuda.synchronize()
    warm_gpu()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for g in graphs:
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    dev_s = e0.elapsed_time(e1) / 1e3
    logical = int(lens_all.astype(np.int64).sum())
    found = np.nonzero(mism.cpu().numpy())[0]
    exact = np.array_equal(found, bad) and int(cnt.sum().item()) == bad.size
    # sampled oracle parity of the recomputed values
    samp = rng.choice(n_total, 200, replace=False)
    comp_h = comp.cpu().numpy().astype(np.uint32)
    ok = True
    for i in samp:
        o, l = int(offs_all[i]), int(lens_all[i])
        ok = ok and oracle.crc32c_raw(arena[o:o + l].cpu().numpy()) == int(comp_h[i])
    emit({"config": "d5 KVCache read-verify (BASELINE configs[4])", "blocks": n_total, "batch": batch,
          "block_sizes_kib": [4, 8, 16, 32, 64], "logical_bytes": logical,
          "blocks_per_s": round(n_total / dev_s), "gbs": round(logical / dev_s / 1e9, 1),
          "frac_hbm": round(logical / dev_s / 1e9 / PEAK, 4), "ms_total": round(dev_s * 1e3, 2),
          "graph_replays": nb, "injected": int(bad.size), "mismatch_set_exact": bool(exact),
          "bit_exact_sample": bool(ok),
          "cpu": cpu_d5() if os.environ.get("SUITE_CPU", "1") == "1" else None})


def _records(cls, n):
    return torch.zeros(n * ctypes.sizeof(cls), dtype=torch.uint8, device=DEV)


def f3_scrub(n=4096, chunk=4 << 20, steps=10, warmup=2, corrupt_frac=1e-3):
    rng = np.random.default_rng(13)
    s = torch.cuda.current_stream()
    data = torch.empty(n * chunk, dtype=torch.uint8, device=DEV)
    L.fill_synth(data, chunk, chunk, n, SEED, 0, stream=s)
    raw = torch.zeros(n, dtype=torch.int32, device=DEV)
    L.create_strided(hf.CRC32C, data, chunk, chunk, n, raw, stream=s)
    torch.cuda.synchronize()
    rawh = raw.cpu().numpy().astype(np.uint32)
    dt = np.dtype([("data", "<u8"), ("length", "<u4"), ("type", "u1"), ("fin", "u1"), ("r", "<u2"),
                   ("checksum", "<u4"), ("computed", "<u4"), ("status", "<i4"), ("r2", "<u4")])
    assert dt.itemsize == ctypes.sizeof(L.ScrubIO)
    rec = np.zeros(n, dtype=dt)
    rec["data"] = data.data_ptr() + np.arange(n, dtype=np.uint64) * chunk
    rec["length"] = chunk
    rec["type"] = hf.CRC32C
    rec["fin"] = np.arange(n) % 2  # odd chunks: chunk-engine ChunkMeta (finalized)
    rec["checksum"] = np.where(rec["fin"] == 1, ~rawh, rawh)
    bad = np.sort(rng.choice(n, max(1, int(n * corrupt_frac)), replace=False))
    rec["checksum"][bad] ^= (1 << rng.integers(0, 32, bad.size)).astype(np.uint32)
    d = torch.from_numpy(rec.view(np.uint8).copy()).to(DEV)
    cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
    warm_gpu()
    wall, dev_s = timed(lambda: L.scrub_batch(hf.CRC32C, d, n, chunk, cnt, stream=s), steps, warmup, s)
    out = d.cpu().numpy().view(dt)
    found = np.nonzero(out["status"])[0]
    exact = np.array_equal(found, bad) and int(cnt.item()) == bad.size
    samp = rng.choice(n, 8, replace=False)
    ok = all(oracle.crc32c_raw(data[i * chunk:(i + 1) * chunk].cpu().numpy()) == int(out["computed"][i])
             for i in samp)
    gbs = n * chunk / dev_s / 1e9
    emit({"config": "f3 scrub: stored chunks vs persisted checksums (SURVEY.md f3)", "chunks": n,
          "chunk_bytes": chunk, "gbs": round(gbs, 1), "frac_hbm": round(gbs / PEAK, 4),
          "ms_per_batch": round(dev_s * 1e3, 3), "wall_ms_per_batch": round(wall * 1e3, 3),
          "injected": int(bad.size), "mismatch_set_exact": bool(exact), "bit_exact_sample": bool(ok)})


def f4_frames(n=1_000_000, steps=10, warmup=2, corrupt=500):
    rng = np.random.default_rng(17)
    s = torch.cuda.current_stream()
    pool = [64, 256, 1024, 4096, 16384]
    if os.environ.get("F4_SIZES"):  # A/B: one size class at a time (F4_SIZES=64, F4_N=...)
        pool = [int(x) for x in os.environ["F4_SIZES"].split(",")]
        n = int(os.environ.get("F4_N", n))
    sizes = rng.choice(pool, n).astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    gapb = 8 + (8 if os.environ.get("F4_ALIGN") == "1" else 0)  # A/B: 16-aligned payloads (not the wire layout)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + gapb)
    offs += gapb  # payload offsets; header at offs - 8
    total = int(offs[-1] + sizes[-1])
    buf = torch.empty(total, dtype=torch.uint8, device=DEV)
    L.fill_synth(buf, total - total % 8, total - total % 8, 1, SEED, 7, stream=s)
    dt = np.dtype([("offset", "<u8"), ("size", "<u4"), ("checksum", "<u4"), ("computed", "<u4"),
                   ("status", "<i4")])
    rec = np.zeros(n, dtype=dt)
    rec["offset"], rec["size"] = offs, sizes
    comp = rng.integers(0, 2, n).astype(np.uint32)
    rec["checksum"] = comp  # compressed bit rides in the header checksum
    d = torch.from_numpy(rec.view(np.uint8).copy()).to(DEV)
    cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
    max_size = max(1 << 20, max(pool))
    L.frame_verify_batch(buf, d, n, max_size, cnt, stream=s)  # -> computed = the sender's calcSerde
    torch.cuda.synchronize()
    computed = d.cpu().numpy().view(dt)["computed"].copy()
    hdr = np.zeros(n, dtype=[("ck", "<u4"), ("size", "<u4")])
    hdr["ck"], hdr["size"] = computed, sizes
    idx = (offs - 8)[:, None] + np.arange(8, dtype=np.uint64)[None, :]
    buf[torch.from_numpy(idx.reshape(-1).view(np.int64)).to(DEV)] = torch.from_numpy(hdr.view(np.uint8)).to(DEV)
    bad = np.sort(rng.choice(n, min(corrupt, max(1, n // 2)), replace=False))
    pos = (offs[bad] + rng.integers(0, sizes[bad])).astype(np.int64)
    buf[torch.from_numpy(pos).to(DEV)] ^= 1
    # host framing walk (Processor::unpackMsg) over the received bytes
    host = buf.cpu().numpy()
    fr = (L.Frame * n)()
    nf, used = ctypes.c_uint64(), ctypes.c_uint64()
    t0 = time.perf_counter()
    rc = L.load().hf3fs_crc_frame_walk(host.ctypes.data, total, fr, n, ctypes.byref(nf), ctypes.byref(used))
    walk_s = time.perf_counter() - t0
    if gapb == 8:  # the wire layout: the walk recovers every frame
        assert rc == 0 and nf.value == n and used.value == total
        d = torch.frombuffer(bytearray(memoryview(fr).cast("B")), dtype=torch.uint8).to(DEV)
    else:  # padded A/B layout: the records as built
        rec["checksum"] = computed
        d = torch.from_numpy(rec.view(np.uint8).copy()).to(DEV)
    warm_gpu()  # (the host framing walk above idles the GPU for ~130 ms)
    wall, dev_s = timed(lambda: L.frame_verify_batch(buf, d, n, max_size, cnt, stream=s), steps, warmup, s)
    out = d.cpu().numpy().view(dt)
    found = np.nonzero(out["status"])[0]
    exact = np.array_equal(found, bad) and int(cnt.item()) == bad.size
    samp = rng.choice(n, min(300, n), replace=False)
    ok = all(oracle.calc_serde(host[int(offs[i]):int(offs[i]) + int(sizes[i])], bool(comp[i])) ==
             int(out["computed"][i]) for i in samp)
    payload = int(sizes.astype(np.int64).sum())
    emit({"config": "f4 serde frame verify (SURVEY.md f4)", "frames": n, "frame_sizes": pool,
          "payload_bytes": payload, "frames_per_s": round(n / dev_s), "gbs": round(payload / dev_s / 1e9, 1),
          "frac_hbm": round(payload / dev_s / 1e9 / PEAK, 4), "ms_per_batch": round(dev_s * 1e3, 3),
          "host_walk_frames_per_s": round(n / walk_s), "injected": int(bad.size),
          "mismatch_set_exact": bool(exact), "bit_exact_sample": bool(ok)})


def f2_coalescer(threads=32, seconds=2.0):
    """Per-IO checksum calls from `threads` threads (tests/cpp/bench_coalescer)."""
    import subprocess
    exe = os.path.join(REPO, "tests", "cpp", "bench_coalescer")
    rows = []
    for mode, t in [("cpu", threads), ("cpu", 1), ("direct-hbm", threads), ("coalesced-hbm", threads),
                    ("coalesced-hbm", 1), ("coalesced-reg", threads), ("coalesced-copy", threads),
                    ("service-hbm", threads), ("service-hbm", 1), ("service-reg", threads), ("service-copy", threads)]:
        r = subprocess.run([exe, "--mode", mode, "--threads", str(t), "--seconds", str(seconds)], capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            raise RuntimeError(f"bench_coalescer {mode}: rc={r.returncode} {r.stderr[-2000:]}")
        rows.append(json.loads(r.stdout.strip().splitlines()[-1]))
    emit({"config": "f2 per-IO read-path checksums, {4..64} KiB blocks, C++ threads (SURVEY.md f2)",
          "results": rows, "bit_exact": all(x["bad"] == 0 for x in rows)})


def f2_read_batch(threads=32, seconds=2.0):
    """The read-path integration INTEGRATION.md 2.1 recommends, at 3FS's call shape: 32
    AioReadWorker threads each reap a batch of completed reads (AioReadWorker.cc:60-94; batch
    reads split at 1024, StorageOperator.cc:163-167) and run setResult's checksum part
    (BatchReadJob.cc:24-63) for the batch -- on the host CPU (the reference, oracle SSE4.2) or as
    one hf3fs_crc_read_result_batch call over registered host memory (gpu-reg) or HBM (gpu-hbm).
    The GPU legs wait with hf3fs_crc_stream_wait (polled, 20 us sleeps): 32 spinning waits on the
    box's 16-CPU quota were throttled by the cgroup (profiles/r05_f2r_matrix.jsonl)."""
    import subprocess
    exe = os.path.join(REPO, "tests", "cpp", "bench_read_batch")
    rows = []
    for batch in (32, 256, 1024):
        for mode in ("cpu", "gpu-reg", "gpu-hbm"):
            r = subprocess.run([exe, "--mode", mode, "--threads", str(threads), "--batch", str(batch), "--seconds",
                                str(seconds), "--wait", "yield"], capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise RuntimeError(f"bench_read_batch {mode} {batch}: rc={r.returncode} {r.stderr[-2000:]}")
            rows.append(json.loads(r.stdout.strip().splitlines()[-1]))
    emit({"config": "f2r read-result batches per reaped AIO batch, {4..64} KiB reads, 32 C++ threads "
                    "(AioReadWorker.cc:60-94, BatchReadJob.cc:24-63)",
          "results": rows, "bit_exact": all(x["bad"] == 0 for x in rows)})


# ------------------------------------------------------------------------------------------
def a2_combine(n=16 << 20, reps=10):
    """A2: element-wise ChecksumInfo::combine (Common.h:179-198) -- the append-write and
    split-read merges -- over n (acc, crc2, len2) triples, len2 uniform in [0, 64 MiB] (1 in 64
    zero: a no-op).  GPU: hf3fs_crc_combine_batch (CRC32C), HIP events; parity and CPU baseline:
    the oracle's C combine over the same triples on every core of the quota."""
    rng = np.random.default_rng(43)
    acc = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    crc2 = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    len2 = rng.integers(0, (64 << 20) + 1, n, dtype=np.uint64)
    len2[::64] = 0
    s = torch.cuda.current_stream()
    d_acc0 = torch.from_numpy(acc.view(np.int32).copy()).to(DEV)
    d_acc = d_acc0.clone()
    d_crc2 = torch.from_numpy(crc2.view(np.int32).copy()).to(DEV)
    d_len2 = torch.from_numpy(len2.view(np.int64).copy()).to(DEV)
    fn = lambda: L.combine_batch(hf.CRC32C, d_acc, d_crc2, d_len2, n, stream=s)  # noqa: E731
    warm_gpu(0.05)
    wall, dev_s = timed(fn, reps, 2, s)
    d_acc.copy_(d_acc0)
    fn()
    got = d_acc.cpu().numpy().view(np.uint32)
    cpus = cpu_cores()
    t0 = time.perf_counter()
    ref = oracle.combine_batch(acc, crc2, len2, threads=cpus["usable"])
    cpu_s = time.perf_counter() - t0
    emit({"config": "A2 combine_batch: element-wise ChecksumInfo::combine (Common.h:179-198)", "n": n,
          "len2": "U[0, 64 MiB], 1/64 zero", "ms_per_batch": round(dev_s * 1e3, 4), "combines_per_s": round(n / dev_s),
          "bit_exact": bool(np.array_equal(got, ref)),
          "cpu": {"label": f"CPU ({cpus['usable']} cores)", "combines_per_s": round(n / cpu_s), "cores": cpus["usable"],
                  "kind": "port", "sample": f"the same {n} triples, oracle/crc_oracle.c orc_combine_batch"},
          "note": "GF(2) algebra on 16-byte triples, VALU-bound: combines/s is the figure"})


# ------------------------------------------------------------------------------------------
def f1_digest(n_files=50_000, blocks_per_file=64, block_len=4 << 20, cpu_files=4_000, reps=10):
    """f1: the admin `checksum` fold (FileWrapper.cc:119-164) over per-chunk read checksums:
    n_files files of blocks_per_file 4 MiB chunks, 5 % short reads (holes zero-filled), 1 %
    missing chunks; both modes (--fill-zero, and strict: the first missing / short chunk is the
    file's status).  GPU: hf3fs_crc_file_digest_batch over the whole table, HIP events.  CPU:
    the oracle's C fold (the reference's work: holes hashed as real zero bytes) on the first
    cpu_files files, every core of the quota; those files are also the parity check."""
    rng = np.random.default_rng(41)
    nb = n_files * blocks_per_file
    blocks = np.zeros(nb, dtype=oracle.BLOCK_DIGEST_DT)
    blocks["block_len"] = block_len
    u = rng.random(nb)
    short = u < 0.05
    missing = (u >= 0.05) & (u < 0.06)
    blocks["read_len"] = np.where(short, rng.integers(0, block_len, nb), block_len)
    blocks["read_len"][missing] = 0
    blocks["missing"] = missing
    blocks["type"] = np.where(missing, 0, 1)
    blocks["checksum"] = np.where(missing, 0, rng.integers(0, 1 << 32, nb, dtype=np.uint64)).astype(np.uint32)
    off = (np.arange(n_files + 1, dtype=np.uint64) * blocks_per_file)
    s = torch.cuda.current_stream()
    d_blocks = torch.from_numpy(blocks.view(np.uint8).copy()).to(DEV)
    d_off = torch.from_numpy(off.view(np.int64).copy()).to(DEV)
    fdt = np.dtype([("length", "<u8"), ("value", "<u4"), ("type", "u1"), ("res", "u1", (3,)), ("status", "<i4"),
                    ("res2", "<u4")])
    d_out = torch.zeros(n_files * fdt.itemsize, dtype=torch.uint8, device=DEV)
    cpus = cpu_cores()
    res = {}
    for fill_zero in (True, False):
        fn = lambda: L.file_digest_batch(d_blocks, d_off, d_out, n_files, blocks_per_file, stream=s,  # noqa: E731
                                         fill_zero=fill_zero)
        warm_gpu(0.05)
        wall, dev_s = timed(fn, reps, 2, s)
        got = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=fdt)
        t0 = time.perf_counter()
        ref = oracle.file_digest_batch(blocks[:cpu_files * blocks_per_file], off[:cpu_files + 1], fill_zero=fill_zero,
                                       threads=cpus["usable"])
        cpu_s = time.perf_counter() - t0
        g = got[:cpu_files]
        exact = bool(np.array_equal(g["status"], ref["status"]) and
                     np.array_equal(np.where(ref["status"] == 0, g["type"], 0), ref["type"]) and
                     np.array_equal(np.where(ref["status"] == 0, g["value"], 0), ref["value"]) and
                     np.all(got["length"] == blocks_per_file * block_len))
        res["fill_zero" if fill_zero else "strict"] = {
            "ms_per_batch": round(dev_s * 1e3, 4), "files_per_s": round(n_files / dev_s),
            "blocks_per_s": round(nb / dev_s), "statuses": {int(k): int(v) for k, v in
                                                            zip(*np.unique(got["status"], return_counts=True))},
            "bit_exact_vs_oracle_files": cpu_files if exact else 0,
            "cpu": {"label": f"CPU ({cpus['usable']} cores)", "files_per_s": round(cpu_files / cpu_s),
                    "blocks_per_s": round(cpu_files * blocks_per_file / cpu_s), "cores": cpus["usable"], "kind": "port",
                    "sample": f"the first {cpu_files} files, oracle/crc_oracle.c orc_file_digest_batch (holes hashed "
                              f"as zero bytes, as FileWrapper.cc:151-153)"}}
    emit({"config": "f1 file digest (admin checksum fold, FileWrapper.cc:119-164; SURVEY.md f1)", "files": n_files,
          "blocks_per_file": blocks_per_file, "block_len": block_len, "short_reads": 0.05, "missing": 0.01,
          "results": res, "bit_exact": all(r["bit_exact_vs_oracle_files"] == cpu_files for r in res.values()),
          "note": "latency-bound GF(2) algebra on 24-byte records (no roofline): blocks/s is the figure"})


if __name__ == "__main__":
    L.load()
    which = sys.argv[1:] or ["d3", "d4", "d5", "a2", "f1", "f2", "f2r", "f3", "f4"]
    for w in which:
        {"d3": d3_ragged, "d4": d4_node, "d5": d5_kv, "a2": a2_combine, "f1": f1_digest, "f2": f2_coalescer,
         "f2r": f2_read_batch, "f3": f3_scrub, "f4": f4_frames}[w]()
        torch.cuda.empty_cache()
