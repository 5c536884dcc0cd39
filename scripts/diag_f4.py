#!/usr/bin/env python3
"""Why the suite's f4 number differs from the in-process A/B: the suite's exact batch
(tests/bench_suite.py f4_frames: real headers, 500 corrupted bytes, records from the host
walk) timed as the suite times it (10 calls after 2 warm-ups, one event pair) and as the
A/B times it (rounds of 5 calls, median), then the same with the A/B's records (all-zero
header checksums), through the Python wrapper and through ctypes directly."""
import ctypes
import importlib
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
lib = L.load()
DEV = torch.device("cuda:0")
s = torch.cuda.current_stream()
rng = np.random.default_rng(17)
n = 1_000_000
pool = [64, 256, 1024, 4096, 16384]
sizes = rng.choice(pool, n).astype(np.uint32)
offs = np.zeros(n, dtype=np.uint64)
offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 8)
offs += 8
total = int(offs[-1] + sizes[-1])
buf = torch.empty(total, dtype=torch.uint8, device=DEV)
L.fill_synth(buf, total - total % 8, total - total % 8, 1, 0x3F5C3C00, 7, stream=s)
dt = np.dtype([("offset", "<u8"), ("size", "<u4"), ("checksum", "<u4"), ("computed", "<u4"), ("status", "<i4")])
rec = np.zeros(n, dtype=dt)
rec["offset"], rec["size"] = offs, sizes
comp = rng.integers(0, 2, n).astype(np.uint32)
rec["checksum"] = comp
d0 = torch.from_numpy(rec.view(np.uint8).copy()).to(DEV)
cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
max_size = 1 << 20
L.frame_verify_batch(buf, d0, n, max_size, cnt, stream=s)
torch.cuda.synchronize()
computed = d0.cpu().numpy().view(dt)["computed"].copy()
real = rec.copy()
real["checksum"] = computed
d_real = torch.from_numpy(real.view(np.uint8).copy()).to(DEV)
d_zero = torch.from_numpy(rec.view(np.uint8).copy()).to(DEV)
sp = ctypes.c_void_p(s.cuda_stream)


def suite_style(fn, steps=10, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(steps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def ab_style(fn, rounds=8, reps=5):
    out = []
    for _ in range(rounds):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / reps)
    return statistics.median(out)


cases = {
    "real_headers_wrapper": lambda: L.frame_verify_batch(buf, d_real, n, max_size, cnt, stream=s),
    "real_headers_ctypes": lambda: lib.hf3fs_crc_frame_verify_batch(buf.data_ptr(), d_real.data_ptr(), n, max_size,
                                                                    cnt.data_ptr(), sp),
    "zero_headers_ctypes": lambda: lib.hf3fs_crc_frame_verify_batch(buf.data_ptr(), d_zero.data_ptr(), n, max_size,
                                                                    cnt.data_ptr(), sp),
}
for rnd in range(2):
    for name, fn in cases.items():
        print(f"round {rnd} {name}: suite-style {suite_style(fn):.4f} ms  ab-style {ab_style(fn):.4f} ms", flush=True)
