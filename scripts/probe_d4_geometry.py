#!/usr/bin/env python3
"""d4 geometry (probe, not product code): is the 64 MiB-chunk cost the
chunk geometry, the footprint, or the code path?  One 64 GiB buffer, one process, cases
interleaved (median of rounds of 3 launches each):
  g64x1024   1024 x 64 MiB create_strided   byte runs: wave w reads [16w, 16w + 16) MiB
  g16x4096   4096 x 16 MiB create_strided   whole buffers: the SAME wave -> address map
  g4x16384   16384 x 4 MiB create_strided   whole buffers, 4 per wave (64 GiB)
  g4x4096    4096 x 4 MiB (first 16 GiB)    bench.py's shape
  g64x256    256 x 64 MiB (first 16 GiB)    byte runs, 4 MiB per wave (r04_d4_tlb's case)
  g64x1024_seg  1024 x 64 MiB as 4 MiB segment tasks (option seg_kib=4096)
The first two touch the same bytes in the same wave order: a gap between them is the code
path (segment shift + atomic vs whole-buffer init), not the geometry.  Digests of the 64 GiB
cases are checked against each other through the combine identity (no oracle here).
PROBE_CASES selects cases; PROBE_ROUNDS rounds."""
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
MIB = 1 << 20
total = 64 << 30
buf = torch.empty(total, dtype=torch.uint8, device=dev)
L.fill_synth(buf, 64 * MIB, 64 * MIB, 1024, 0x3F5C3C00, 0, stream=s)
cases = {
    "g64x1024": (1024, 64, None),
    "g16x4096": (4096, 16, None),
    "g4x16384": (16384, 4, None),
    "g4x4096": (4096, 4, None),
    "g64x256": (256, 64, None),
    "g64x1024_seg": (1024, 64, "4096"),
}
want = os.environ.get("PROBE_CASES")
if want:
    cases = {k: v for k, v in cases.items() if k in want.split(",")}
outs = {k: torch.zeros(v[0], dtype=torch.int32, device=dev) for k, v in cases.items()}


def run(k):
    n, mib, seg = cases[k]
    if seg:
        L.set_option("seg_kib", seg)
    L.create_strided(hf.CRC32C, buf, mib * MIB, mib * MIB, n, outs[k], stream=s)
    if seg:
        L.set_option("seg_kib", "0")


res = {k: [] for k in cases}
for rnd in range(int(os.environ.get("PROBE_ROUNDS", 5))):
    for k in cases:
        run(k)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(3):
            run(k)
        b.record(s)
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) / 3)
# consistency: a 64 MiB chunk's raw CRC from its four 16 MiB parts (each hashed from ~0):
# raw(A||B) = raw(A) x^(8|B|) ^ raw(B, 0), raw(B, 0) = raw(B, ~0) ^ ~0 x^(8|B|)
agree = None
if "g64x1024" in outs and "g16x4096" in outs:
    c64 = outs["g64x1024"].cpu().numpy().view(np.uint32)
    c16 = outs["g16x4096"].cpu().numpy().view(np.uint32)
    agree = True
    for i in (0, 511, 1023):
        v = int(c16[4 * i])
        for j in range(1, 4):
            v = L.crc32c_combine(v, int(c16[4 * i + j]), 16 * MIB) ^ L.shift(hf.CRC32C, 0xFFFFFFFF, 16 * MIB)
        agree = agree and v == int(c64[i])
for k, v in res.items():
    n, mib, seg = cases[k]
    ms = statistics.median(v)
    print(json.dumps({"probe": "d4_geometry", "case": k, "chunks": n, "chunk_mib": mib, "seg_kib": seg,
                      "footprint_gib": n * mib / 1024, "ms": round(ms, 4), "tbs": round(n * mib * MIB / ms / 1e9, 3),
                      "runs": [round(x, 4) for x in v]}), flush=True)
print(json.dumps({"probe": "d4_geometry", "combine_check": agree}), flush=True)
