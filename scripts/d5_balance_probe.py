#!/usr/bin/env python3
"""Probe: is d5 limited by per-wave work imbalance?  Same bytes per batch,
block sizes random over {4..64} KiB (d5) vs all 24 KiB vs all 64 KiB, timed
with HIP events on one stream (verify_blocks, computed given)."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hf = importlib.import_module("3fs_amd")
L = hf._lib
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
arena_bytes = 32 << 30
arena = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)
L.fill_synth(arena, 1 << 30, 1 << 30, 32, 0x3F5C3C00, 0, stream=s)
rng = np.random.default_rng(5)
total = 1_000_000 * 24.8 * 1024
for name, sizes in [("mixed", None), ("u24", 24), ("u64", 64), ("u4", 4)]:
    if sizes is None:
        lens = (rng.choice([4, 8, 16, 32, 64], 1_000_000) * 1024).astype(np.uint32)
    else:
        n = int(total // (sizes * 1024))
        lens = np.full(n, sizes * 1024, dtype=np.uint32)
    n = lens.size
    offs = (rng.integers(0, (arena_bytes - 65536) // 4096, n) * 4096).astype(np.uint64)
    O = torch.tensor(offs.view(np.int64), device=dev)
    Ls = torch.tensor(lens.view(np.int32), device=dev)
    exp = torch.zeros(n, dtype=torch.int32, device=dev)
    comp = torch.zeros(n, dtype=torch.int32, device=dev)
    mism = torch.zeros(n, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    f = lambda: L.verify_blocks(hf.CRC32C, arena, O, Ls, exp, mism, cnt, n, 65536, computed=comp, stream=s)  # noqa
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        f()
    e1.record()
    torch.cuda.synchronize()
    sec = e0.elapsed_time(e1) / 1e3 / 10
    print(f"{name}: blocks {n} bytes {int(lens.astype(np.int64).sum())} -> {lens.astype(np.int64).sum() / sec / 1e9:.1f} GB/s, {sec * 1e3:.3f} ms", flush=True)
