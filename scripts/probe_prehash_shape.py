#!/usr/bin/env python3
"""Which property of the d3 pre-hash job list costs rate?  (probe, not product code)

The pre hash (payload + old-byte ranges of 4096 updates, byte runs) reads ~3.96 GB about 6 %
slower than the same bytes as equal contiguous ranges.  One process, one buffer set, every
case through create_batch with option list_runs=1 (the update pipeline's byte-run schedule),
interleaved over rounds (median):
  equal     8192 equal 1 KiB-aligned ranges, back to back        (the bulk-like baseline)
  unalign   the same, every start moved by a random 0..127 bytes  (unaligned starts)
  spread    the same equal ranges, one per 2 MiB slot of the 16 GiB chunk buffer
  ragged    the pre-hash job lengths, back to back, 1 KiB-aligned starts
  ragged_u  the pre-hash job lengths, back to back, byte-packed (unaligned starts)
  jobs      the pre-hash job list itself (payload + old bytes interleaved)
  jobs_sort the same jobs sorted by address (payload region first)
Prints one JSON line per case: median ms, TB/s, rounds."""
import importlib
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hf = importlib.import_module("3fs_amd")
L = hf._lib
L.load()
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
n, chunk = 4096, 4 << 20
rng = np.random.default_rng(3)
sizes = rng.integers(2 << 20, chunk + 1, n).astype(np.int64)
lens = rng.integers(64 << 10, (1 << 20) + 1, n)
offs = np.array([rng.integers(0, chunk - ln + 1) for ln in lens])
old = np.clip(np.minimum(offs + lens, sizes) - offs, 0, None)
chunks = torch.empty(n * chunk, dtype=torch.uint8, device=dev)
L.fill_synth(chunks, chunk, chunk, n, 0x3F5C3C00, 0, stream=s)
payload = torch.empty(n * (1 << 20), dtype=torch.uint8, device=dev)
L.fill_synth(payload, 1 << 20, 1 << 20, n, 0x3F5C3C00 ^ 0xABCD, 0, stream=s)
pa = payload.data_ptr() + np.arange(n, dtype=np.uint64) * (1 << 20)
oa = chunks.data_ptr() + np.arange(n, dtype=np.uint64) * chunk + offs.astype(np.uint64)
ja = np.empty(2 * n, dtype=np.uint64)
jl = np.empty(2 * n, dtype=np.int64)
ja[0::2], ja[1::2] = pa, oa
jl[0::2], jl[1::2] = lens, old
total = int(jl.sum())
base = chunks.data_ptr()
eq = (total // (2 * n)) // 1024 * 1024


def lst(addrs, ls):
    A = torch.tensor(np.asarray(addrs, dtype=np.uint64).view(np.int64), device=dev)
    Ln = torch.tensor(np.asarray(ls, dtype=np.int64), device=dev)
    out = torch.zeros(len(ls), dtype=torch.int32, device=dev)
    return (lambda: L.create_batch(1, A, Ln, out, len(ls), int(max(ls)), stream=s)), int(np.sum(ls))


def packed(ls, align):
    a = np.zeros(len(ls), dtype=np.uint64)
    p = 0
    for i, x in enumerate(ls):
        a[i] = base + p
        p += int(x)
        p = (p + align - 1) // align * align
    return a


cases = {
    "equal": lst(base + np.arange(2 * n, dtype=np.uint64) * eq, [eq] * (2 * n)),
    "unalign": lst(base + np.arange(2 * n, dtype=np.uint64) * (eq + 128) + rng.integers(0, 128, 2 * n).astype(np.uint64),
                   [eq] * (2 * n)),
    "spread": lst(base + np.arange(2 * n, dtype=np.uint64) * (2 << 20), [eq] * (2 * n)),
    "ragged": lst(packed(jl, 1024), jl),
    "ragged_u": lst(packed(jl, 1), jl),
    "jobs": lst(ja, jl),
}
p = np.argsort(ja, kind="stable")
cases["jobs_sort"] = lst(ja[p], jl[p])
if os.environ.get("PROBE_PARTS") == "1":  # each region alone vs its lengths packed / slot-aligned
    m = old > 0
    mean = int(lens.mean()) // 1024 * 1024
    cases = {
        "pay": lst(pa, lens),
        "pay_packed": lst(packed(lens, 1024), lens),
        "pay_eq_slots": lst(pa, [mean] * n),
        "old": lst(oa[m], old[m]),
        "old_packed": lst(packed(old[m], 1024), old[m]),
        "old_at_chunk_start": lst(chunks.data_ptr() + np.nonzero(m)[0].astype(np.uint64) * chunk, old[m]),
        "old_1k_aligned": lst((oa[m] // 1024) * 1024, old[m]),
    }
reps = {}
if os.environ.get("PROBE_WIN") == "1":  # windows: option prehash_rep runs per wave (list_runs honours it)
    base_cases = {k: cases[k] for k in ("ragged_u", "jobs", "jobs_sort")}
    cases = {}
    for k, c in base_cases.items():
        for r in (1, 2, 4):
            cases[f"{k}_rep{r}"] = c
            reps[f"{k}_rep{r}"] = r
L.set_option("list_runs", "1")
res = {k: [] for k in cases}
for rnd in range(int(os.environ.get("ROUNDS", 7))):
    for k, (fn, nb) in cases.items():
        L.set_option("prehash_rep", str(reps.get(k, 1)))
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / 5)
L.set_option("list_runs", "0")
for k, (fn, nb) in cases.items():
    ms = statistics.median(res[k])
    print(json.dumps({"probe": "prehash_shape", "case": k, "bytes": nb, "ms": round(ms, 4), "tbs": round(nb / ms / 1e9, 3),
                      "runs": [round(x, 4) for x in res[k]]}), flush=True)
