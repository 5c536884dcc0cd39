#!/usr/bin/env python3
"""Randomized soak of the HIP path against the oracle (test infrastructure, not collected by
pytest): `python tests/soak.py SECONDS [SEED]`.

Every round draws a fresh configuration and checks every result bit for bit:
  * update batches (hf3fs_crc_update_batch): 8-96 chunks of 512 B .. 2 MiB, writes / truncates /
    extends with random offsets, 5 % corrupted client checksums, DELTA or REFERENCE, the
    three-pass or the fused pipeline, apply pieces down to 1 KiB, scratch poisoned or not,
    on the null stream or a side stream -- state carried across rounds per chunk set, as the
    replica oracle (ChunkReplica::update restated, oracle/oracle.py replica_apply) carries it;
    statuses, checksum cases, sizes, checksums and chunk bytes compared, and the library's
    self-check record (hf3fs_crc_anomalies) must stay empty;
  * create batches (hf3fs_crc_create_batch): 1-20 k ranges of 0..300 KB at every alignment,
    random start values, CRC32C or CRC32, planner tasks or byte runs (option list_runs);
  * KV-block verify (hf3fs_crc_verify_blocks) with injected mismatches: exact mismatch set.
Prints a progress line about every 20 s and one JSON summary line; exit status 1 on any
mismatch.  The round-4 incident is the reason it exists: it turns GPU minutes
into many independent seeds of the paths that once returned a wrong checksum."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
hf = importlib.import_module("3fs_amd")
import oracle as orc  # noqa: E402

orc.lib()
L = hf._lib
dev = torch.device("cuda:0")
secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60
seed = int(sys.argv[2]) if len(sys.argv) > 2 else int(time.time()) & 0xFFFF
rng = np.random.default_rng(seed)
side = torch.cuda.Stream(dev)
stats = {"seed": seed, "update_rounds": 0, "update_ios": 0, "create_batches": 0, "create_ranges": 0,
         "verify_batches": 0, "verify_blocks": 0, "failures": []}


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def fail(kind, detail):
    stats["failures"].append({"kind": kind, "detail": detail})
    print("FAIL", kind, detail, flush=True)


class ChunkSet:
    """n chunks of chunk_size on the device and their oracle replicas."""

    def __init__(self, n, cs):
        self.n, self.cs = n, cs
        self.chunks = [bytearray(cs) for _ in range(n)]
        self.sizes, self.cks = [0] * n, [(1, 0)] * n
        self.d = torch.zeros(n * cs, dtype=torch.uint8, device=dev)
        self.payload = torch.zeros(n * cs, dtype=torch.uint8, device=dev)


def random_ios(cs_, mixed):
    ios = []
    for c in range(cs_.n):
        r = rng.random()
        if mixed and r < 0.08:
            ios.append(("T", int(rng.integers(0, cs_.cs + 1))))
        elif mixed and r < 0.12:
            ios.append(("E", int(rng.integers(0, cs_.cs + 1))))
        else:
            off = cs_.sizes[c] if r < 0.3 else int(rng.integers(0, cs_.cs))
            if off >= cs_.cs:
                off = int(rng.integers(0, cs_.cs))
            ln = int(rng.integers(1, cs_.cs - off + 1))
            ln = min(ln, max(1, int(rng.integers(1, cs_.cs // 2 + 2))))
            ios.append(("W", off, ln))
    return ios


def update_round(cs_):
    mode = int(rng.integers(0, 2))
    pipeline = ["mode", "unfused", "fused"][int(rng.integers(0, 3))]
    fine = rng.random() < 0.3
    poison = rng.random() < 0.2
    on_side = rng.random() < 0.5
    # the three-pass pipeline's apply: ticketed tasks (fine: up to 65 pieces of >= 1 KiB), or the
    # one-shot apply (auto / always / a 256-workgroup grid that loops) with 4, 8 or 16 KiB pieces
    grid = "0" if fine else ["-1", "0", "1", "2"][int(rng.integers(0, 4))]
    piece = ["4", "8", "16"][int(rng.integers(0, 3))]
    L.set_option("update_pipeline", pipeline)
    L.set_option("apply_pieces", "64" if fine else "8")
    L.set_option("apply_min_kib", "1" if fine else "64")
    L.set_option("apply_grid", grid)
    L.set_option("apply_piece_kib", piece)
    L.set_option("poison", str(0xA5A5A5A5 if poison else 0))
    n, cs = cs_.n, cs_.cs
    ios = random_ios(cs_, rng.random() < 0.5)
    arr = (hf.UpdateIO * n)()
    host_payload = np.zeros(n * cs, dtype=np.uint8)
    expect = []
    for c, io in enumerate(ios):
        u = arr[c]
        u.chunk = cs_.d.data_ptr() + c * cs
        u.chunk_size = cs_.sizes[c]
        u.chunk_checksum_type, u.chunk_checksum = cs_.cks[c]
        if io[0] == "W":
            _, off, ln = io
            data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            host_payload[c * cs:c * cs + ln] = np.frombuffer(data, np.uint8)
            wck = orc.create(1, data)
            if rng.random() < 0.05:
                wck = (1, wck[1] ^ 0x10)
            u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
            u.payload = cs_.payload.data_ptr() + c * cs
            u.write_checksum_type, u.write_checksum = wck
            expect.append(orc.replica_apply(cs_.chunks[c], cs_.sizes[c], cs_.cks[c], orc.WRITE, off, ln, data, wck,
                                            with_case=True))
        else:
            kind = hf.UPDATE_TRUNCATE if io[0] == "T" else hf.UPDATE_EXTEND
            u.update_type, u.offset, u.length = kind, 0, int(io[1])
            expect.append(orc.replica_apply(cs_.chunks[c], cs_.sizes[c], cs_.cks[c], kind, 0, int(io[1]),
                                            with_case=True))
    cs_.payload.copy_(to_dev(host_payload))
    d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
    torch.cuda.synchronize()
    L.anomalies(reset=True)
    if on_side:
        with torch.cuda.stream(side):
            L.update_batch(1, d_ios, n, cs, mode=mode, stream=side)
    else:
        L.update_batch(1, d_ios, n, cs, mode=mode, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
    hchunks = cs_.d.cpu().numpy()
    cfg = {"mode": mode, "pipeline": pipeline, "fine": fine, "poison": poison, "side": on_side, "cs": cs,
           "apply_grid": grid, "apply_piece_kib": piece}
    for c in range(n):
        rc, size, ck, kase = expect[c]
        got = (res[c].status, res[c].checksum_case, res[c].out_size, res[c].out_checksum_type, res[c].out_checksum)
        if got != (rc, kase, size, ck[0], ck[1]):
            fail("update", {**cfg, "io": [str(x) for x in ios[c]], "got": got, "want": (rc, kase, size) + tuple(ck)})
        elif bytes(hchunks[c * cs:c * cs + size]) != bytes(cs_.chunks[c][:size]):
            fail("update_bytes", {**cfg, "io": [str(x) for x in ios[c]]})
        cs_.sizes[c], cs_.cks[c] = size, tuple(ck)
    rec = L.anomalies(reset=True)
    if rec.get("count"):
        fail("anomaly", {**cfg, "record": rec})
    L.set_option("poison", "0")
    stats["update_rounds"] += 1
    stats["update_ios"] += n


def create_round(host, arena):
    n = int(rng.integers(1, 20_000))
    ctype = int(rng.integers(1, 3))
    runs = rng.random() < 0.5
    maxl = int(rng.choice([40, 4096, 70_000, 300_000]))
    lens = rng.integers(0, maxl + 1, n)
    offs = rng.integers(0, host.size - maxl - 1, n)
    starts = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    L.set_option("list_runs", "1" if runs else "0")
    A = torch.tensor((np.uint64(arena.data_ptr()) + offs.astype(np.uint64)).view(np.int64), device=dev)
    Ls = torch.tensor(lens.astype(np.int64), device=dev)
    S = torch.tensor(starts.view(np.int32), device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    L.create_batch(ctype, A, Ls, out, n, max(1, int(lens.max())), starts=S, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    L.set_option("list_runs", "0")
    got = u32(out)
    raw = orc.crc32c_raw if ctype == 1 else orc.crc32_raw
    for i in range(n):
        want = raw(host[int(offs[i]):int(offs[i]) + int(lens[i])], int(starts[i]))
        if int(got[i]) != want:
            fail("create", {"ctype": ctype, "runs": runs, "i": i, "off": int(offs[i]), "len": int(lens[i])})
            break
    stats["create_batches"] += 1
    stats["create_ranges"] += n


def verify_round(host, arena):
    m = int(rng.integers(1000, 200_000))
    kl = rng.choice([4096, 8192, 16384, 32768, 65536], m).astype(np.uint32)
    ko = (rng.integers(0, (host.size - 65536) // 4096, m) * 4096).astype(np.uint64)
    exp = np.array([orc.crc32c_raw(host[int(o):int(o) + int(l)]) for o, l in zip(ko, kl)], dtype=np.uint32)
    bad = np.sort(rng.choice(m, min(50, m), replace=False))
    exp[bad] ^= 1
    mism = torch.zeros(m, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    L.verify_blocks(1, arena, to_dev(ko.view(np.int64)), to_dev(kl.view(np.int32)), to_dev(exp.view(np.int32)),
                    mism, cnt, m, 65536, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    found = np.nonzero(mism.cpu().numpy())[0]
    if not np.array_equal(found, bad) or int(cnt.item()) != bad.size:
        fail("verify", {"m": m, "found": int(found.size), "want": int(bad.size)})
    stats["verify_batches"] += 1
    stats["verify_blocks"] += m


def main():
    size = 64 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host)
    sets = [ChunkSet(int(rng.integers(8, 97)), int(rng.choice([512, 4096, 65536, 128 << 10, 1 << 20, 2 << 20])))
            for _ in range(4)]
    t0 = last = time.time()
    k = 0
    while time.time() - t0 < secs and len(stats["failures"]) < 20:
        r = k % 4
        if r < 2:
            update_round(sets[int(rng.integers(0, len(sets)))])
        elif r == 2:
            create_round(host, arena)
        else:
            verify_round(host, arena)
        k += 1
        if time.time() - last > 20:
            last = time.time()
            print(json.dumps({"t": round(last - t0), **{k2: v for k2, v in stats.items() if k2 != "failures"},
                              "failures": len(stats["failures"])}), flush=True)
    stats["seconds"] = round(time.time() - t0, 1)
    print(json.dumps({"soak": "done", **stats}), flush=True)
    return 1 if stats["failures"] else 0


if __name__ == "__main__":
    sys.exit(main())
