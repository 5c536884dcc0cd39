#!/usr/bin/env python3
"""d4 HBM-resident rate vs the planner's task size: 1024 x 64 MiB create_strided,
HIP events over 5 launches after 2 warm-ups; HF3FS_CRC_SEG_KIB overrides the
segment size (unset: the planner's choice)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hf = importlib.import_module("3fs_amd")
L = hf._lib
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
n, chunk = int(os.environ.get("D4_N", 1024)), 64 << 20
buf = torch.empty(n * chunk, dtype=torch.uint8, device=dev)
L.fill_synth(buf, chunk, chunk, n, 0x3F5C3C00, 0, stream=s)
out = torch.zeros(n, dtype=torch.int32, device=dev)
for _ in range(2):
    L.create_strided(hf.CRC32C, buf, chunk, chunk, n, out, stream=s)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    L.create_strided(hf.CRC32C, buf, chunk, chunk, n, out, stream=s)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(f"d4 seg_kib={os.environ.get('HF3FS_CRC_SEG_KIB', 'plan')} n={n} {n * chunk / ms / 1e9:.1f} TB/s {ms:.3f} ms")
