#!/usr/bin/env python3
"""Where does the d3 pre-hash lose bandwidth? (probe, not product code)  The DELTA pre-hash
reads every payload and the old bytes under it (~3.9-4.2 GB per batch) at ~5.0 TB/s while the
bulk create runs 6.7.  Same plan as tests/bench_suite.py d3 (first batch), hashed with
create_batch over: the payload ranges alone, the old-byte ranges alone, both interleaved (the
pre-hash's job list), and the whole payload buffer as 4096 x 1 MiB strided."""
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


def timed(fn, reps=10):
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
    return lambda: L.create_batch(1, A, Ln, out, len(ls), mx, stream=s), int(np.sum(ls))


inter_a = np.empty(2 * n, dtype=np.uint64)
inter_l = np.empty(2 * n, dtype=np.int64)
inter_a[0::2], inter_a[1::2] = pa, oa
inter_l[0::2], inter_l[1::2] = lens, old
cases = {"payload_ranges": lst(pa, lens), "old_ranges": lst(oa[old > 0], old[old > 0]),
         "interleaved_prehash_jobs": lst(inter_a, inter_l)}
out = torch.zeros(n, dtype=torch.int32, device=dev)
cases["payload_buffer_strided_1MiB"] = (lambda: L.create_strided(1, payload, 1 << 20, 1 << 20, n, out, stream=s),
                                        n << 20)
for seg in os.environ.get("SEG_SWEEP", "").split(",") if os.environ.get("SEG_SWEEP") else [None]:
    if seg is not None:
        L.set_option("seg_kib", seg)
    for name, (fn, nbytes) in cases.items():
        ms = timed(fn)
        print(json.dumps({"probe": "d3_prehash", "seg_kib": seg, "case": name, "bytes": nbytes, "ms": round(ms, 4),
                          "tbs": round(nbytes / ms / 1e9, 3)}), flush=True)
