#!/usr/bin/env python3
"""verify_blocks over one block size (D5_KIB, all blocks) or the d5 mix (D5_KIB unset),
~25 GB per batch, timed with HIP events: the per-task cost probe for PMC passes."""
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
kib = os.environ.get("D5_KIB")
total = 1_000_000 * 24.8 * 1024
if kib:
    n = int(total // (int(kib) * 1024))
    lens = np.full(n, int(kib) * 1024, dtype=np.uint32)
else:
    lens = (rng.choice([4, 8, 16, 32, 64], 1_000_000) * 1024).astype(np.uint32)
n = lens.size
offs = (rng.integers(0, (arena_bytes - 65536) // 4096, n) * 4096).astype(np.uint64)
O = torch.tensor(offs.view(np.int64), device=dev)
Ls = torch.tensor(lens.view(np.int32), device=dev)
exp = torch.zeros(n, dtype=torch.int32, device=dev)
mism = torch.zeros(n, dtype=torch.uint8, device=dev)
cnt = torch.zeros(1, dtype=torch.int32, device=dev)
comp = torch.zeros(n, dtype=torch.int32, device=dev)
for _ in range(2):
    L.verify_blocks(1, arena, O, Ls, exp, mism, cnt, n, 65536, computed=comp, stream=s)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    L.verify_blocks(1, arena, O, Ls, exp, mism, cnt, n, 65536, computed=comp, stream=s)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 3
print(f"d5 probe kib={kib or 'mix'} blocks={n} {lens.astype(np.int64).sum() / ms / 1e9:.1f} TB/s {ms:.3f} ms")
