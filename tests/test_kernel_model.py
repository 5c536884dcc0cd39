"""CPU model of the k_crc_ranges algebra (3fs_amd/csrc/crc_kernels.hip), checked
against the oracle.  Pins the stream layout (lane l, dword d of each 1 KiB
block), the per-stream step s <- (s ^ w) * x^8192, the fold tree, the virtual
alignment/masking and the final x^(8e - 8160) shift -- without a GPU."""
import random

import numpy as np
import pytest

M32 = 0xFFFFFFFF


def gf(orc, a, b, poly):
    return orc.lib().orc_gf2_mulmod(a & M32, b & M32, poly)


def xpow_bits(orc, e, poly):
    """x^e for signed e using x^-1 = (poly << 1) | 1."""
    if e >= 0:
        base, n = 0x40000000, e
    else:
        base, n = ((poly << 1) | 1) & M32, -e
    r = 0x80000000
    while n:
        if n & 1:
            r = gf(orc, r, base, poly)
        base = gf(orc, base, base, poly)
        n >>= 1
    return r


def model_range(orc, mem, a0, a1, poly):
    """hash_range(): returns (V, vend)."""
    vs = a0 & ~15
    nb = (a1 - vs + 1023) // 1024
    k8192 = xpow_bits(orc, 8192, poly)
    s = np.zeros((64, 4), dtype=np.uint64)
    for b in range(nb):
        for lane in range(64):
            g = vs + b * 1024 + 16 * lane
            gran = bytes(mem[x] if a0 <= x < a1 else 0 for x in range(g, g + 16))
            for d in range(4):
                w = int.from_bytes(gran[4 * d:4 * d + 4], "little")
                s[lane, d] = gf(orc, int(s[lane, d]) ^ w, k8192, poly)
    x32 = xpow_bits(orc, 32, poly)
    u = []
    for lane in range(64):
        v = gf(orc, int(s[lane, 0]), x32, poly) ^ int(s[lane, 1])
        v = gf(orc, v, x32, poly) ^ int(s[lane, 2])
        v = gf(orc, v, x32, poly) ^ int(s[lane, 3])
        u.append(v)
    for k in range(6):  # shuffle tree
        step = 1 << k
        xl = xpow_bits(orc, 128 << k, poly)
        for lane in range(0, 64, 2 * step):
            u[lane] = gf(orc, u[lane], xl, poly) ^ u[lane + step]
    return u[0], vs + nb * 1024


def model_create(orc, mem, base, length, start, seg_bytes, poly):
    acc = 0
    segs = max(1, (length + seg_bytes - 1) // seg_bytes)
    for seg in range(segs):
        tb = seg * seg_bytes
        if seg and tb >= length:
            continue
        te = min(length, tb + seg_bytes)
        v, ebits = 0, 0
        if te > tb:
            v, vend = model_range(orc, mem, base + tb, base + te, poly)
            ebits = 8 * (base + length - vend) - 8160
        val = gf(orc, v, xpow_bits(orc, ebits, poly), poly)
        if seg == 0:
            val ^= gf(orc, start, xpow_bits(orc, 8 * length, poly), poly)
        acc ^= val
    return acc


@pytest.mark.parametrize("align,length,seg", [(0, 1024, 1024), (3, 1, 1024), (5, 2047, 1024), (15, 3000, 2048),
                                              (0, 0, 1024), (8, 5000, 1024), (0, 4096, 4096), (1, 17, 1024)])
def test_model_matches_oracle(orc, align, length, seg):
    rnd = random.Random(length * 31 + align)
    base = 4096 + align
    mem = {base + i: rnd.getrandbits(8) for i in range(length)}
    data = bytes(mem[base + i] for i in range(length))
    for poly, fn in [(orc.POLY_CRC32C, orc.crc32c_raw), (orc.POLY_CRC32, orc.crc32_raw)]:
        for start in (M32, 0, 0x1234567):
            assert model_create(orc, mem, base, length, start, seg, poly) == fn(data, start)
