#!/usr/bin/env python3
"""d4 (1024 x 64 MiB, 64 GiB HBM-resident) runs ~6 % below d2 (4096 x 4 MiB, 16 GiB) on the
same box.  Geometry or allocation?  (probe, not product code)
One process; each case = 3 create_strided launches timed with HIP events, one JSON line:
  big_d4      1024 x 64 MiB over a 64 GiB allocation (the suite's d4)
  big_d2_lo   4096 x 4 MiB over the first 16 GiB of that allocation
  big_d2_hi   4096 x 4 MiB over its last 16 GiB
  small_d2    4096 x 4 MiB over a fresh 16 GiB allocation (bench.py's d2)
  small_d4    256 x 64 MiB over that 16 GiB allocation
Run plain for the rates, and under rocprofv3 --pmc (UTCL1 translation counters; FETCH_SIZE) for
per-dispatch counters: dispatches come in the order above, 3 per case after 1 warm-up each."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hf = importlib.import_module("3fs_amd")
L = hf._lib
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
MiB, GiB = 1 << 20, 1 << 30


def case(name, base, chunk, n, reps=3):
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    L.create_strided(hf.CRC32C, base, chunk, chunk, n, out, stream=s)  # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        L.create_strided(hf.CRC32C, base, chunk, chunk, n, out, stream=s)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"probe": "d4_tlb", "case": name, "chunks": n, "chunk_mib": chunk // MiB,
                      "ms": round(ms, 4), "tbs": round(n * chunk / ms / 1e9, 3)}), flush=True)


big = torch.empty(64 * GiB, dtype=torch.uint8, device=dev)
L.fill_synth(big, 64 * MiB, 64 * MiB, 1024, 0x3F5C3C00, 0, stream=s)
case("big_d4", big, 64 * MiB, 1024)
case("big_d2_lo", big, 4 * MiB, 4096)
case("big_d2_hi", big.data_ptr() + 48 * GiB, 4 * MiB, 4096)
del big
torch.cuda.empty_cache()
small = torch.empty(16 * GiB, dtype=torch.uint8, device=dev)
L.fill_synth(small, 4 * MiB, 4 * MiB, 4096, 0x3F5C3C00, 0, stream=s)
case("small_d2", small, 4 * MiB, 4096)
case("small_d4", small, 64 * MiB, 256)
