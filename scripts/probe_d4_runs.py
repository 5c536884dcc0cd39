#!/usr/bin/env python3
"""d4 geometry as byte runs (probe, not product code): 1024 x 64 MiB HBM-resident chunks hashed
by create_strided (the planner: 4 MiB segments on a static stride) against the same chunks as
a create_batch list with option list_runs = 1 (each wave one exact 16 MiB share) and = 0,
interleaved in one process, median of rounds; digests must agree."""
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
n, ch = int(os.environ.get("D4_N", 1024)), 64 << 20
buf = torch.empty(n * ch, dtype=torch.uint8, device=dev)
L.fill_synth(buf, ch, ch, n, 0x3F5C3C00, 0, stream=s)
A = torch.tensor((buf.data_ptr() + np.arange(n, dtype=np.uint64) * ch).view(np.int64), device=dev)
Ln = torch.full((n,), ch, dtype=torch.int64, device=dev)
outs = {k: torch.zeros(n, dtype=torch.int32, device=dev) for k in ("strided", "runs", "tasks")}


def run(k):
    if k == "strided":
        L.create_strided(hf.CRC32C, buf, ch, ch, n, outs[k], stream=s)
    else:
        L.set_option("list_runs", "1" if k == "runs" else "0")
        L.create_batch(hf.CRC32C, A, Ln, outs[k], n, ch, stream=s)
        L.set_option("list_runs", "0")


res = {k: [] for k in outs}
for rnd in range(6):
    for k in outs:
        run(k)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(3):
            run(k)
        b.record(s)
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) / 3)
ref = outs["strided"].cpu()
for k, v in res.items():
    ms = statistics.median(v)
    print(json.dumps({"probe": "d4_runs", "case": k, "ms": round(ms, 4), "tbs": round(n * ch / ms / 1e9, 3),
                      "agree": bool(torch.equal(outs[k].cpu(), ref))}), flush=True)
