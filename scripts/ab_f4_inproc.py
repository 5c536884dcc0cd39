#!/usr/bin/env python3
"""Interleaved in-process A/B of f4 frame verification across library builds.

Loads every 3fs_amd/lib/ab/NAME.so of AB_LIBS into ONE process (ctypes, no
package import) and times hf3fs_crc_frame_verify_batch of each on the SAME
device buffer and frame records, interleaved over rounds, so buffer placement
and clock drift are shared by all variants.  Sizes: F4_SIZES (comma list),
F4_N frames.  Prints median / min ms per batch per build and whether every
build's computed values and mismatch count agree with the first one's.
"""
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
names = os.environ.get("AB_LIBS", "head_u4").split()
# AB_ENV="option=a,b,c": one library, variants = values of a library option (hf3fs_crc_set_option)
env_var, env_vals = None, []
if os.environ.get("AB_ENV"):
    env_var, vals = os.environ["AB_ENV"].split("=")
    env_vals = vals.split(",")
    names = [f"{names[0]}@{v}" for v in env_vals]
libs = {}
for nm in names:
    if "@" in nm:
        base = nm.split("@")[0]
        if base + "@" + env_vals[0] != nm:
            libs[nm] = libs[base + "@" + env_vals[0]]
            continue
        nm_file = base
    else:
        nm_file = nm
    lib = ctypes.CDLL(os.path.join(REPO, "3fs_amd", "lib", "ab", nm_file + ".so"), mode=ctypes.RTLD_LOCAL)
    lib.hf3fs_crc_frame_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_void_p, ctypes.c_void_p]
    lib.hf3fs_crc_fill_synth.argtypes = [ctypes.c_void_p] + [ctypes.c_uint64] * 5 + [ctypes.c_void_p]
    lib.hf3fs_crc_set_option.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libs[nm] = lib
pool = [int(x) for x in os.environ.get("F4_SIZES", "64,256,1024,4096,16384").split(",")]
n = int(os.environ.get("F4_N", 1_000_000))
rng = np.random.default_rng(17)
sizes = rng.choice(pool, n).astype(np.uint32)
offs = np.zeros(n, dtype=np.uint64)
offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 8)
offs += 8
total = int(offs[-1] + sizes[-1])
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
sp = ctypes.c_void_p(s.cuda_stream)
buf = torch.empty(total, dtype=torch.uint8, device=dev)
first = libs[names[0]]
assert first.hf3fs_crc_fill_synth(buf.data_ptr(), total - total % 8, total - total % 8, 1, 0x3F5C3C00, 7, sp) == 0
dt = np.dtype([("offset", "<u8"), ("size", "<u4"), ("checksum", "<u4"), ("computed", "<u4"), ("status", "<i4")])
rec = np.zeros(n, dtype=dt)
rec["offset"], rec["size"] = offs, sizes
d = torch.from_numpy(rec.view(np.uint8).copy()).to(dev)
cnt = torch.zeros(1, dtype=torch.int32, device=dev)
max_size = max(1 << 20, max(pool))


def run(lib, nm=None):
    if env_var and nm:
        assert lib.hf3fs_crc_set_option(env_var.encode(), nm.split("@")[1].encode()) == 0
    assert lib.hf3fs_crc_frame_verify_batch(buf.data_ptr(), d.data_ptr(), n, max_size, cnt.data_ptr(), sp) == 0


run(first, names[0])
torch.cuda.synchronize()
ref = d.cpu().numpy().view(dt)["computed"].copy()
res = {k: [] for k in names}
agree = {k: True for k in names}
for rnd in range(int(os.environ.get("AB_ROUNDS", 6))):
    for nm in names if rnd % 2 == 0 else names[::-1]:
        lib = libs[nm]
        run(lib, nm)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run(lib, nm)
        e1.record()
        torch.cuda.synchronize()
        res[nm].append(e0.elapsed_time(e1) / 5)
        got = d.cpu().numpy().view(dt)["computed"]
        agree[nm] = agree[nm] and bool(np.array_equal(got, ref)) and int(cnt.item()) == n  # every header is 0: all mismatch
payload = int(sizes.astype(np.int64).sum())
for nm in names:
    med = statistics.median(res[nm])
    print(f"{nm}: median {med:.3f} ms min {min(res[nm]):.3f} ms  {payload / med / 1e9:.1f} GB/s  agree={agree[nm]}")
