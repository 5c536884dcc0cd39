#!/usr/bin/env python3
"""Interleaved in-process A/B of k_crc_ranges across library builds (AB_LIBS,
3fs_amd/lib/ab/NAME.so): d2 (create_strided, 4096 x 4 MiB) and d5
(verify_blocks, 1M KV blocks of {4..64} KiB at 4 KiB-aligned offsets of a
32 GiB arena).  Same buffers for every build; rounds alternate the order.
AB_CASES selects ("d2 d5"); "pre" = the d3 DELTA pre-hash job list (payload + old-byte ranges
of tests/bench_suite.py d3's first batch) as byte runs (option list_runs), create_batch."""
import ctypes
import os
import statistics

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
names = os.environ.get("AB_LIBS", "base").split()
cases = os.environ.get("AB_CASES", "d2 d5").split()
V, U64, U32, U8 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint8
libs = {}
for nm in names:
    lib = ctypes.CDLL(os.path.join(REPO, "3fs_amd", "lib", "ab", nm + ".so"), mode=ctypes.RTLD_LOCAL)
    lib.hf3fs_crc_create_strided.argtypes = [U8, V, U64, U64, U64, U32, V, V]
    lib.hf3fs_crc_verify_blocks.argtypes = [U8, V, V, V, V, V, V, V, U64, U32, V]
    lib.hf3fs_crc_fill_synth.argtypes = [V, U64, U64, U64, U64, U64, V]
    lib.hf3fs_crc_create_batch.argtypes = [U8, V, V, V, V, U64, U64, V]
    lib.hf3fs_crc_set_option.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libs[nm] = lib
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
sp = ctypes.c_void_p(s.cuda_stream)
first = libs[names[0]]


def bench(run, check, rounds=6, reps=5):
    res = {k: [] for k in names}
    ok = {k: True for k in names}
    run(first)
    torch.cuda.synchronize()
    ref = check()
    for rnd in range(rounds):
        for nm in names if rnd % 2 == 0 else names[::-1]:
            run(libs[nm])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run(libs[nm])
            e1.record()
            torch.cuda.synchronize()
            res[nm].append(e0.elapsed_time(e1) / reps)
            ok[nm] = ok[nm] and np.array_equal(check(), ref)
    return res, ok


if "d2" in cases:
    n, L = 4096, 4 << 20
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    assert first.hf3fs_crc_fill_synth(buf.data_ptr(), L, L, n, 0x3F5C3C00, 0, sp) == 0
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    res, ok = bench(lambda lib: lib.hf3fs_crc_create_strided(1, buf.data_ptr(), L, L, n, 0xFFFFFFFF, out.data_ptr(), sp),
                    lambda: out.cpu().numpy().copy())
    for nm in names:
        med = statistics.median(res[nm])
        print(f"d2 {nm}: median {med:.4f} ms min {min(res[nm]):.4f}  {n * L / med / 1e9:.1f} TB/s  agree={ok[nm]}")
    del buf
    torch.cuda.empty_cache()
for case in [c for c in cases if c.startswith("d5")]:  # d5: the {4..64} KiB mix; d5uK: all K KiB
    rng = np.random.default_rng(5)
    arena_bytes = 32 << 30
    arena = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)
    assert first.hf3fs_crc_fill_synth(arena.data_ptr(), 1 << 30, 1 << 30, 32, 0x3F5C3C00, 0, sp) == 0
    n = 1_000_000
    lens = (rng.choice([4, 8, 16, 32, 64], n) * 1024).astype(np.uint32)
    if case != "d5":
        kib = int(case[3:])
        n = int(lens.astype(np.int64).sum() // (kib * 1024))
        lens = np.full(n, kib * 1024, dtype=np.uint32)
    offs = (rng.integers(0, (arena_bytes - 65536) // 4096, n) * 4096).astype(np.uint64)
    O = torch.tensor(offs.view(np.int64), device=dev)
    Ls = torch.tensor(lens.view(np.int32), device=dev)
    exp = torch.zeros(n, dtype=torch.int32, device=dev)
    mism = torch.zeros(n, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    comp = torch.zeros(n, dtype=torch.int32, device=dev)
    res, ok = bench(lambda lib: lib.hf3fs_crc_verify_blocks(1, arena.data_ptr(), O.data_ptr(), Ls.data_ptr(),
                                                            exp.data_ptr(), mism.data_ptr(), cnt.data_ptr(),
                                                            comp.data_ptr(), n, 65536, sp),
                    lambda: comp.cpu().numpy().copy())
    del arena
    tot = int(lens.astype(np.int64).sum())
    for nm in names:
        med = statistics.median(res[nm])
        print(f"{case} {nm}: median {med:.4f} ms min {min(res[nm]):.4f}  {tot / med / 1e9:.1f} TB/s  agree={ok[nm]}")

if "pre" in cases:
    rng = np.random.default_rng(3)
    n, chunk = 4096, 4 << 20
    sizes = rng.integers(2 << 20, chunk + 1, n).astype(np.int64)
    lens = rng.integers(64 << 10, (1 << 20) + 1, n)
    offs = np.array([rng.integers(0, chunk - ln + 1) for ln in lens])
    r = rng.random(n)
    app = (r < 0.10) & (sizes + lens <= chunk)
    offs[app] = sizes[app]
    old = np.clip(np.minimum(offs + lens, sizes) - offs, 0, None)
    chunks = torch.empty(n * chunk, dtype=torch.uint8, device=dev)
    assert first.hf3fs_crc_fill_synth(chunks.data_ptr(), chunk, chunk, n, 0x3F5C3C00, 0, sp) == 0
    payload = torch.empty(n << 20, dtype=torch.uint8, device=dev)
    assert first.hf3fs_crc_fill_synth(payload.data_ptr(), 1 << 20, 1 << 20, n, 0x3F5C3C00 ^ 0xABCD, 0, sp) == 0
    a = np.empty(2 * n, dtype=np.uint64)
    ln = np.empty(2 * n, dtype=np.int64)
    a[0::2] = payload.data_ptr() + np.arange(n, dtype=np.uint64) * (1 << 20)
    a[1::2] = chunks.data_ptr() + np.arange(n, dtype=np.uint64) * chunk + offs.astype(np.uint64)
    ln[0::2], ln[1::2] = lens, old
    A = torch.tensor(a.view(np.int64), device=dev)
    Ln = torch.tensor(ln, device=dev)
    out = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    for lib in libs.values():
        assert lib.hf3fs_crc_set_option(b"list_runs", b"1") == 0
    res, ok = bench(lambda lib: lib.hf3fs_crc_create_batch(1, A.data_ptr(), Ln.data_ptr(), None, out.data_ptr(), 2 * n,
                                                           int(ln.max()), sp),
                    lambda: out.cpu().numpy().copy())
    total = int(ln.sum())
    for nm in names:
        med = statistics.median(res[nm])
        print(f"pre {nm}: median {med:.4f} ms min {min(res[nm]):.4f}  {total / med / 1e9:.1f} TB/s  agree={ok[nm]}")
