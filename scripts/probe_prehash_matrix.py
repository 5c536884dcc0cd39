#!/usr/bin/env python3
"""Where does a ragged range list lose against the uniform bulk stream?  (probe, not product code)

The d3 DELTA pre hash reads ~4 GB of payload and old-byte ranges at ~5.1 TB/s; the bulk create
of 4096 x 1 MiB runs 6.6.  One process, one set of buffers, the plan of tests/bench_suite.py
d3's first batch; every case hashes through the public ABI (create_batch / create_strided),
with option list_runs selecting the byte-run schedule the update pipeline uses:
  A uniform: payload buffer as 4096 x 1 MiB strided (whole-buffer tasks)
  B payload ranges (U[64 KiB, 1 MiB] at 1 MiB-aligned slots): planner tasks / byte runs
  C old-byte ranges (unaligned, inside 4 MiB chunks): planner / byte runs
  D the pre hash's job list (payload and old bytes interleaved): planner / byte runs
  E the same byte count as ONE contiguous range: byte runs (no range boundary at all)
  F the same byte count as 8192 equal contiguous 1 KiB-aligned ranges: byte runs
Prints one JSON line per case: ms (HIP events, mean of reps after a warm-up) and TB/s."""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hf = importlib.import_module("3fs_amd")
L = hf._lib
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
n, chunk = 4096, 4 << 20
reps = int(os.environ.get("REPS", 10))
rng = np.random.default_rng(3)
sizes = rng.integers(2 << 20, chunk + 1, n).astype(np.int64)
lens = rng.integers(64 << 10, (1 << 20) + 1, n)
offs = np.array([rng.integers(0, chunk - ln + 1) for ln in lens])
r = rng.random(n)
app = (r < 0.10) & (sizes + lens <= chunk)
offs[app] = sizes[app]
old = np.clip(np.minimum(offs + lens, sizes) - offs, 0, None)
chunks = torch.empty(n * chunk, dtype=torch.uint8, device=dev)
L.fill_synth(chunks, chunk, chunk, n, 0x3F5C3C00, 0, stream=s)
payload = torch.empty(n * (1 << 20), dtype=torch.uint8, device=dev)
L.fill_synth(payload, 1 << 20, 1 << 20, n, 0x3F5C3C00 ^ 0xABCD, 0, stream=s)
pa = payload.data_ptr() + np.arange(n, dtype=np.uint64) * (1 << 20)
oa = chunks.data_ptr() + np.arange(n, dtype=np.uint64) * chunk + offs.astype(np.uint64)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def lst(addrs, ls):
    A = torch.tensor(np.asarray(addrs, dtype=np.uint64).view(np.int64), device=dev)
    Ln = torch.tensor(np.asarray(ls, dtype=np.int64), device=dev)
    out = torch.zeros(len(ls), dtype=torch.int32, device=dev)
    mx = int(max(ls))
    return (lambda: L.create_batch(1, A, Ln, out, len(ls), mx, stream=s)), int(np.sum(ls)), out


inter_a = np.empty(2 * n, dtype=np.uint64)
inter_l = np.empty(2 * n, dtype=np.int64)
inter_a[0::2], inter_a[1::2] = pa, oa
inter_l[0::2], inter_l[1::2] = lens, old
total = int(inter_l.sum())
# E / F: the same byte count, contiguous, from the start of the chunk buffer
contig = lst([chunks.data_ptr()], [total])
eq = (total // (2 * n)) // 1024 * 1024
equal = lst(chunks.data_ptr() + np.arange(2 * n, dtype=np.uint64) * eq, [eq] * (2 * n))
out = torch.zeros(n, dtype=torch.int32, device=dev)
cases = [("A_uniform_strided_1MiB", None, (lambda: L.create_strided(1, payload, 1 << 20, 1 << 20, n, out, stream=s),
                                           n << 20, out))]
for name, c in [("B_payload_ranges", lst(pa, lens)), ("C_old_ranges", lst(oa[old > 0], old[old > 0])),
                ("D_prehash_jobs", lst(inter_a, inter_l))]:
    cases += [(name + "_tasks", "0", c), (name + "_runs", "1", c)]
cases += [("E_one_contiguous_range_runs", "1", contig), ("F_equal_contiguous_ranges_runs", "1", equal),
          ("F_equal_contiguous_ranges_tasks", "0", equal)]
# G: the job list as byte runs right after a 2.2 GB device copy (the previous batch's apply in
# d3: its stores are still being written back when the next pre hash starts); only the hash
# is timed, per launch, between events recorded after the copy
cpy_src = payload[:2200 << 20]
cpy_dst = chunks[8 << 30:(8 << 30) + (2200 << 20)]


def after_copy(fn):
    ms = []
    for _ in range(reps + 1):
        cpy_dst.copy_(cpy_src)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return sum(ms[1:]) / reps


check = {}
for rnd in range(int(os.environ.get("ROUNDS", 2))):
    for name, runs, (fn, nbytes, o) in cases:
        if runs is not None:
            L.set_option("list_runs", runs)
        ms = timed(fn)
        L.set_option("list_runs", "0")
        digest = int(o.cpu().numpy().astype(np.uint32).astype(np.uint64).sum())
        key = name.rsplit("_", 1)[0]
        same = check.setdefault(key, digest) == digest  # tasks and runs give the same digests
        print(json.dumps({"probe": "prehash_matrix", "round": rnd, "case": name, "bytes": nbytes, "ms": round(ms, 4),
                          "tbs": round(nbytes / ms / 1e9, 3), "same_digests": same}), flush=True)
    fn, nbytes, o = cases[[c[0] for c in cases].index("D_prehash_jobs_runs")][2]
    L.set_option("list_runs", "1")
    ms = after_copy(fn)
    L.set_option("list_runs", "0")
    print(json.dumps({"probe": "prehash_matrix", "round": rnd, "case": "G_prehash_jobs_runs_after_2200MB_copy",
                      "bytes": nbytes, "ms": round(ms, 4), "tbs": round(nbytes / ms / 1e9, 3)}), flush=True)
