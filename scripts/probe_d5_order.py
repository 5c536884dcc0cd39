#!/usr/bin/env python3
"""d5 block order (probe, not product code): does the address order of KV blocks in a verify
batch set its rate?  The d5 shape -- 1M blocks of {4..64} KiB at 4 KiB-aligned random offsets
of a 32 GiB arena -- verified (verify_blocks, d_computed given) as drawn, sorted by offset,
and with the offsets confined to windows of W GiB of the arena (blocks drawn per window),
interleaved in one process, median of rounds.  Every case checks its mismatch count (no
flips: 0).  PROBE_ROUNDS rounds."""
import importlib
import json
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
hf = importlib.import_module("3fs_amd")
L = hf._lib
L.load()
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
GIB = 1 << 30
arena_gib = 32
arena = torch.empty(arena_gib * GIB, dtype=torch.uint8, device=dev)
L.fill_synth(arena, GIB, GIB, arena_gib, 0x3F5C3C00, 0, stream=s)
rng = np.random.default_rng(5)
n = 1_000_000
lens = (rng.choice([4, 8, 16, 32, 64], n) * 1024).astype(np.uint32)
offs = (rng.integers(0, (arena_gib * GIB - 65536) // 4096, n) * 4096).astype(np.uint64)


def case_arrays(order):
    if order == "drawn":
        return offs, lens
    if order == "sorted":
        p = np.argsort(offs, kind="stable")
        return offs[p], lens[p]
    w = int(order[len("window"):])  # blocks grouped by w GiB windows, random order within each
    key = offs // np.uint64(w * GIB)
    p = np.argsort(key, kind="stable")
    return offs[p], lens[p]


cases = {}
for order in ("drawn", "sorted", "window4", "window16"):
    o, ln = case_arrays(order)
    O = torch.tensor(o.view(np.int64), device=dev)
    Ls = torch.tensor(ln.view(np.int32), device=dev)
    addrs = torch.tensor((o + np.uint64(arena.data_ptr())).view(np.int64), device=dev)
    exp = torch.zeros(n, dtype=torch.int32, device=dev)
    L.create_batch(hf.CRC32C, addrs, Ls.to(torch.int64), exp, n, 65536, stream=s)
    cases[order] = (O, Ls, exp, torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros(1, dtype=torch.int32, device=dev),
                    torch.zeros(n, dtype=torch.int32, device=dev))
torch.cuda.synchronize()
total = int(lens.astype(np.int64).sum())
res = {k: [] for k in cases}
for rnd in range(int(os.environ.get("PROBE_ROUNDS", 7))):
    for k, (O, Ls, exp, mism, cnt, comp) in cases.items():
        L.verify_blocks(hf.CRC32C, arena, O, Ls, exp, mism, cnt, n, 65536, computed=comp, stream=s)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(3):
            L.verify_blocks(hf.CRC32C, arena, O, Ls, exp, mism, cnt, n, 65536, computed=comp, stream=s)
        b.record(s)
        torch.cuda.synchronize()
        assert int(cnt.item()) == 0, k
        res[k].append(a.elapsed_time(b) / 3)
for k, v in res.items():
    ms = statistics.median(v)
    print(json.dumps({"probe": "d5_order", "case": k, "blocks": n, "bytes": total, "ms": round(ms, 4),
                      "tbs": round(total / ms / 1e9, 3), "runs": [round(x, 4) for x in v]}), flush=True)
