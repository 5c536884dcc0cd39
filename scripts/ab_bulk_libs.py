#!/usr/bin/env python3
"""Interleaved in-process A/B of hf3fs_crc_create_strided across library builds (probe).

Loads every 3fs_amd/lib/ab/NAME.so of AB_LIBS into ONE process (ctypes) and times the d2
bulk launch (AB_N x AB_LEN, default 4096 x 4 MiB) of each on the SAME buffer, interleaved
over AB_ROUNDS rounds of 5 launches (HIP events); prints median / min ms, TB/s and whether
every build's digests equal the first build's."""
import ctypes
import os
import statistics

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
names = os.environ.get("AB_LIBS", "s_off s_on").split()
n, length = int(os.environ.get("AB_N", 4096)), int(os.environ.get("AB_LEN", 4 << 20))
libs = {}
for nm in names:
    lib = ctypes.CDLL(os.path.join(REPO, "3fs_amd", "lib", "ab", nm + ".so"), mode=ctypes.RTLD_LOCAL)
    lib.hf3fs_crc_create_strided.argtypes = [ctypes.c_uint8, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    lib.hf3fs_crc_fill_synth.argtypes = [ctypes.c_void_p] + [ctypes.c_uint64] * 5 + [ctypes.c_void_p]
    libs[nm] = lib
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
sp = ctypes.c_void_p(s.cuda_stream)
buf = torch.empty(n * length, dtype=torch.uint8, device=dev)
assert libs[names[0]].hf3fs_crc_fill_synth(buf.data_ptr(), length, length, n, 0x3F5C3C00, 0, sp) == 0
outs = {k: torch.zeros(n, dtype=torch.int32, device=dev) for k in names}


def run(k):
    assert libs[k].hf3fs_crc_create_strided(1, buf.data_ptr(), length, length, n, 0xFFFFFFFF, outs[k].data_ptr(), sp) == 0


for k in names:
    run(k)
torch.cuda.synchronize()
res = {k: [] for k in names}
for rnd in range(int(os.environ.get("AB_ROUNDS", 9))):
    for k in names if rnd % 2 == 0 else names[::-1]:
        run(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run(k)
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / 5)
ref = outs[names[0]].cpu()
for k in names:
    med = statistics.median(res[k])
    print(f"{k}: median {med:.4f} ms min {min(res[k]):.4f} ms  {n * length / med / 1e9:.1f} GB/s  "
          f"agree={bool(torch.equal(outs[k].cpu(), ref))}", flush=True)
