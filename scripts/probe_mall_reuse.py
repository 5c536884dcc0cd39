#!/usr/bin/env python3
"""Does a payload hashed a moment ago come back from the Infinity Cache (MALL) when it is
copied?  (probe, not product code -- the premise of a d3 schedule that applies each group of
writes right after hashing it, instead of after the whole batch's pre hash)

One process.  For a region of S MiB (the group's payload): hash it (create_strided, loads
non-temporal or cached via option nt), then stream T MiB of other data through the GPU
(interference: the other groups' old bytes and stores), then copy the region to a
destination; only the copy is timed (HIP events around it).  Baseline: the same copy of a
region nobody touched since a 2 GiB sweep (cold).  Prints one JSON line per case."""
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
MiB = 1 << 20
reps = int(os.environ.get("REPS", 6))
src = torch.empty(8 << 30, dtype=torch.uint8, device=dev)
L.fill_synth(src, 1 << 20, 1 << 20, (8 << 30) >> 20, 7, 0, stream=s)
dst = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
sweep = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
junk = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
out = torch.zeros(4096, dtype=torch.int32, device=dev)
torch.cuda.synchronize()


def ev():
    return torch.cuda.Event(enable_timing=True)


def case(S, T, nt, hashed):
    ms = []
    for r in range(reps + 1):
        base = (r % 6) * (1 << 30)  # a different region each rep
        reg = src[base:base + S * MiB]
        sweep.add_(1)  # evict: 2 GiB read + write
        if hashed:
            L.set_option("nt", "1" if nt else "0")
            L.create_strided(1, reg, MiB, MiB, S, out, stream=s)
            L.set_option("nt", "1")
        if T:
            junk[:T * MiB].add_(1)  # T MiB read + written by someone else
        e0, e1 = ev(), ev()
        e0.record()
        dst[:S * MiB].copy_(reg)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    m = sum(ms[1:]) / reps
    print(json.dumps({"probe": "mall_reuse", "S_MiB": S, "T_MiB": T, "hash_loads": ("nt" if nt else "cached") if hashed else "none",
                      "copy_ms": round(m, 4), "copy_tbs_rw": round(2 * S * MiB / m / 1e9, 3)}), flush=True)


for S in (32, 64, 128):
    case(S, 0, True, False)
    for nt in (False, True):
        for T in (0, 32, 64, 128, 256):
            case(S, T, nt, True)
