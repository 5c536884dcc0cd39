#!/usr/bin/env python3
"""Fixed cost per launch of the bulk create kernel (probe, not product code): create_strided
over n x 4 MiB chunks for n = 128 ... 4096, back-to-back launches timed with events (median
of rounds), then a least-squares fit ms = a + bytes / rate.  a is what one launch pays
whatever its size (ramp, tail, gap); the d3 pre hash (3.96 GB) and apply are short enough
for it to matter."""
import importlib
import json
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
hf = importlib.import_module("3fs_amd")
L = hf._lib
L.load()
from bench_suite import warm_gpu  # noqa: E402

dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
CH = 4 << 20
NMAX = 4096
buf = torch.empty(NMAX * CH, dtype=torch.uint8, device=dev)
L.fill_synth(buf, CH, CH, NMAX, 0x3F5C3C00, 0, stream=s)
out = torch.zeros(NMAX, dtype=torch.int32, device=dev)
ns = [int(x) for x in os.environ.get("FC_NS", "128,256,512,1024,2048,4096").split(",")]
reps, rounds = 10, 7
res = {}
for rnd in range(rounds):
    for n in ns:
        warm_gpu(0.02)
        L.create_strided(hf.CRC32C, buf, CH, CH, n, out, stream=s)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            L.create_strided(hf.CRC32C, buf, CH, CH, n, out, stream=s)
        b.record(s)
        torch.cuda.synchronize()
        res.setdefault(n, []).append(a.elapsed_time(b) / reps)
xs, ys = [], []
for n in ns:
    ms = statistics.median(res[n])
    xs.append(n * CH / 1e9)
    ys.append(ms)
    print(json.dumps({"probe": "fixed_cost", "chunks": n, "gb": round(n * CH / 1e9, 3), "ms": round(ms, 4),
                      "tbs": round(n * CH / ms / 1e9, 3)}), flush=True)
A = np.vstack([np.ones(len(xs)), xs]).T
(a0, slope), *_ = np.linalg.lstsq(A, np.array(ys), rcond=None)
print(json.dumps({"probe": "fixed_cost_fit", "fixed_us": round(a0 * 1e3, 1),
                  "marginal_tbs": round(1 / slope, 3)}), flush=True)
