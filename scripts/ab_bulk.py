#!/usr/bin/env python3
"""Interleaved A/B of bulk-path launch variants in ONE process (cdna guide §5.4 rule 24).

Variants toggle the host planner through env vars read at every call:
HF3FS_CRC_SEG_KIB (task size) and HF3FS_CRC_STATIC (no ticket queue).
Prints median / min launch ms per variant over interleaved rounds.
"""
import importlib
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hf = importlib.import_module("3fs_amd")
L = hf._lib
n, length = int(os.environ.get("AB_N", 4096)), int(os.environ.get("AB_LEN", 4 << 20))
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
buf = torch.empty(n * length, dtype=torch.uint8, device=dev)
L.fill_synth(buf, length, length, n, 0x3F5C3C00, 0, stream=s)
out = torch.zeros(n, dtype=torch.int32, device=dev)
variants = {  # library options (hf3fs_crc_set_option)
    "auto": {"nt": "0"},
    "auto_nt": {"nt": "1"},
    "seg1024": {"seg_kib": "1024", "nt": "0"},
    "seg1024_nt": {"seg_kib": "1024", "nt": "1"},
    "direct": {"seg_kib": str(length >> 10), "nt": "0"},
    "direct_nt": {"seg_kib": str(length >> 10), "nt": "1"},
}
if os.environ.get("AB_SEGS"):  # AB_SEGS="0 4096 16384": task sizes in KiB (0 = the planner's), NT loads
    variants = {f"seg{k}": {"seg_kib": k, "nt": "1"} for k in os.environ["AB_SEGS"].split()}
res = {k: [] for k in variants}
ref = None
for rnd in range(5):
    for name, env in variants.items():
        for k, v in {"static": "0", "seg_kib": "0", "nt": "1", **env}.items():
            L.set_option(k, v)
        for _ in range(2):
            L.create_strided(hf.CRC32C, buf, length, length, n, out, stream=s)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(s)
            L.create_strided(hf.CRC32C, buf, length, length, n, out, stream=s)
            b.record(s)
        torch.cuda.synchronize()
        res[name] += [a.elapsed_time(b) for a, b in ev]
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref), name
summary = {k: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
               "gbs_at_median": round(n * length / (statistics.median(v) / 1e3) / 1e9, 1)} for k, v in res.items()}
print(json.dumps(summary, indent=1))
