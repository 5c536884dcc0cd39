#!/usr/bin/env python3
"""Per-part cost of the byte-run schedule (probe, not product code).  The same ~3.96 GB (the d3
pre hash's byte count) as equal, contiguous, 1 KiB-aligned ranges of 4 MiB down to 32 KiB,
hashed through create_batch as byte runs (option list_runs=1, the update pipeline's pre-hash
schedule) and as whole-range tasks (list_runs=0), plus create_strided over the 4 MiB and 1 MiB
layouts (the bench kernel).  A byte run crosses ~ranges / 4096 part boundaries per wave; the
slope of ms over ranges is what one boundary costs the kernel.  One JSON line per case."""
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
TOTAL = 3959 << 20
buf = torch.empty(TOTAL + (4 << 20), dtype=torch.uint8, device=dev)
L.fill_synth(buf, 4 << 20, 4 << 20, (TOTAL >> 22) + 1, 0x3F5C3C00, 0, stream=s)
reps, rounds = 10, 5


def lst(sz):
    k = TOTAL // sz
    A = torch.tensor((buf.data_ptr() + np.arange(k, dtype=np.uint64) * sz).view(np.int64), device=dev)
    Ln = torch.full((k,), sz, dtype=torch.int64, device=dev)
    out = torch.zeros(k, dtype=torch.int32, device=dev)
    return (lambda: L.create_batch(1, A, Ln, out, k, sz, stream=s)), k * sz, out


cases = []
for sz in [int(x) << 10 for x in os.environ.get("PC_KIB", "4096,1024,482,256,128,64,32").split(",")]:
    fn, nbytes, out = lst(sz)
    cases += [(f"runs_{sz >> 10}KiB", "1", fn, nbytes, out), (f"tasks_{sz >> 10}KiB", "0", fn, nbytes, out)]
for sz in (4 << 20, 1 << 20):
    k = TOTAL // sz
    out = torch.zeros(k, dtype=torch.int32, device=dev)
    cases.append((f"strided_{sz >> 10}KiB", None,
                  (lambda sz=sz, k=k, out=out: L.create_strided(1, buf, sz, sz, k, out, stream=s)), k * sz, out))
res, dig = {}, {}
for rnd in range(rounds):
    for name, runs, fn, nbytes, out in cases:
        if runs is not None:
            L.set_option("list_runs", runs)
        warm_gpu(0.02)
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        L.set_option("list_runs", "0")
        res.setdefault(name, []).append(a.elapsed_time(b) / reps)
        d = int(out.cpu().numpy().astype(np.uint32).astype(np.uint64).sum())
        key = name.split("_", 1)[1]
        dig.setdefault(key, set()).add(d)
for name, runs, fn, nbytes, out in cases:
    ms = statistics.median(res[name])
    key = name.split("_", 1)[1]
    print(json.dumps({"probe": "part_cost", "case": name, "gb": round(nbytes / 1e9, 3), "ms": round(ms, 4),
                      "ms_min": round(min(res[name]), 4), "tbs": round(nbytes / ms / 1e9, 3),
                      "digests_agree": len(dig[key]) == 1}), flush=True)
