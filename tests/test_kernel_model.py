"""CPU model of the k_crc_ranges algebra (3fs_amd/csrc/crc_kernels.hip), checked
against the oracle.  Pins, without a GPU: the stream layout (lane l, dword d of
each 1 KiB block), the per-stream step s <- (s ^ w) * x^8192, the fold with
negative-power constants, both block grids (end-aligned for single-task buffers
with the start value xor-ed into the first four bytes; start-aligned for
segmented buffers with the x^(8e) shift and start * x^(8 len) term) and the
masking of bytes outside the buffer."""
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


def model_grid(orc, mem, vs, nb, a0, a1, poly, init=None):
    """hash_grid() + fold_streams(): lin(bytes of [vs, vs + 1024 nb) masked to [a0, a1))."""
    k8192 = xpow_bits(orc, 8192, poly)
    s = np.zeros((64, 4), dtype=np.uint64)
    for b in range(nb):
        for lane in range(64):
            g = vs + b * 1024 + 16 * lane
            gran = bytearray(mem.get(x, 0) if a0 <= x < a1 else 0 for x in range(g, g + 16))
            if init is not None and b == 0:
                o = (a0 - vs) - 16 * lane
                for d in range(4):
                    sh = o - 4 * d
                    if -4 < sh < 4:
                        w = int.from_bytes(gran[4 * d:4 * d + 4], "little")
                        w ^= ((init << (8 * sh)) if sh >= 0 else (init >> (-8 * sh))) & M32
                        gran[4 * d:4 * d + 4] = w.to_bytes(4, "little")
            for d in range(4):
                w = int.from_bytes(gran[4 * d:4 * d + 4], "little")
                s[lane, d] = gf(orc, int(s[lane, d]) ^ w, k8192, poly)
    c0 = xpow_bits(orc, -32, poly)
    u = []
    for lane in range(64):
        v = gf(orc, int(s[lane, 3]), c0, poly) ^ int(s[lane, 2])
        v = gf(orc, v, c0, poly) ^ int(s[lane, 1])
        v = gf(orc, v, c0, poly) ^ int(s[lane, 0])
        u.append(v)
    for k in range(6):
        step = 1 << k
        ck = xpow_bits(orc, -(128 << k), poly)
        for lane in range(0, 64, 2 * step):
            u[lane] ^= gf(orc, u[lane + step], ck, poly)
    return u[0]


def model_direct(orc, mem, base, length, start, poly):
    a0, a1 = base, base + length
    vend = (a1 + 15) & ~15
    nb = (vend - (a0 & ~15) + 1023) // 1024
    vs = vend - nb * 1024
    spill = a0 - vs > 1020  # start bytes would straddle into block 1: explicit start term instead
    r = model_grid(orc, mem, vs, nb, a0, a1, poly, init=start if length >= 4 and not spill else None)
    pad = vend - a1
    if pad:
        r = gf(orc, r, xpow_bits(orc, -8 * pad, poly), poly)
    if length < 4 or spill:
        r ^= gf(orc, start, xpow_bits(orc, 8 * length, poly), poly)
    return r


def model_segmented(orc, mem, base, length, start, seg_bytes, poly):
    acc = 0
    for seg in range(max(1, (length + seg_bytes - 1) // seg_bytes)):
        tb = seg * seg_bytes
        te = min(length, tb + seg_bytes)
        a0, a1 = base + tb, base + te
        vs = a0 & ~15
        nb = (a1 - vs + 1023) // 1024
        v = model_grid(orc, mem, vs, nb, a0, a1, poly)
        val = gf(orc, v, xpow_bits(orc, 8 * (base + length - (vs + nb * 1024)), poly), poly)
        if seg == 0:
            val ^= gf(orc, start, xpow_bits(orc, 8 * length, poly), poly)
        acc ^= val
    return acc


CASES = [(0, 1024), (3, 1), (5, 2047), (15, 3000), (8, 5000), (0, 4096), (1, 17), (12, 4), (13, 5), (2, 3),
         (0, 1040), (7, 1100),
         # start bytes at the end of block 0 (a0 - vs = 1023, 1022, 1021): the spill case
         (15, 1024), (14, 1025), (13, 1027), (15, 8189)]


@pytest.mark.parametrize("align,length", CASES)
def test_model_direct_matches_oracle(orc, align, length):
    rnd = random.Random(length * 31 + align)
    base = 4096 + align
    mem = {base + i: rnd.getrandbits(8) for i in range(length)}
    data = bytes(mem[base + i] for i in range(length))
    for poly, fn in [(orc.POLY_CRC32C, orc.crc32c_raw), (orc.POLY_CRC32, orc.crc32_raw)]:
        for start in (M32, 0, 0x1234567):
            assert model_direct(orc, mem, base, length, start, poly) == fn(data, start)


@pytest.mark.parametrize("align,length,seg", [(0, 4096, 1024), (5, 3000, 2048), (15, 5000, 1024), (1, 17, 1024)])
def test_model_segmented_matches_oracle(orc, align, length, seg):
    rnd = random.Random(length * 7 + align)
    base = 8192 + align
    mem = {base + i: rnd.getrandbits(8) for i in range(length)}
    data = bytes(mem[base + i] for i in range(length))
    for poly, fn in [(orc.POLY_CRC32C, orc.crc32c_raw), (orc.POLY_CRC32, orc.crc32_raw)]:
        for start in (M32, 0x1234567):
            assert model_segmented(orc, mem, base, length, start, seg, poly) == fn(data, start)


def _short_tables(orc, poly):
    """PolyTables::dw (x^32 dword slices), ::b8 (x^8 byte table) as built in hf3fs_crc_api.hip."""
    x32, x8 = xpow_bits(orc, 32, poly), xpow_bits(orc, 8, poly)
    dw = [[gf(orc, b << (8 * k), x32, poly) for b in range(256)] for k in range(4)]
    b8 = [gf(orc, b, x8, poly) for b in range(256)]
    return dw, b8


def model_lin_t(dw, b8, mem, a, b):
    """lin_t() of frame_kernels.hip: bytes [a, b) of the 32-byte window at a & ~15,
    whole dwords through dw, edge bytes through b8."""
    g = a & ~15
    w = [int.from_bytes(bytes(mem.get(g + 4 * k + t, 0) for t in range(4)), "little") for k in range(8)]
    ja, jb, c = a - g, b - g, 0
    for k in range(8):
        lo, hi = max(ja, 4 * k), min(jb, 4 * k + 4)
        if hi - lo == 4:
            c ^= w[k]
            c = dw[0][c & 0xFF] ^ dw[1][(c >> 8) & 0xFF] ^ dw[2][(c >> 16) & 0xFF] ^ dw[3][c >> 24]
        else:
            for t in range(lo - 4 * k, hi - 4 * k):
                c = (c >> 8) ^ b8[(c ^ (w[k] >> (8 * t))) & 0xFF]
    return c


@pytest.mark.parametrize("poly", [0x82F63B78, 0xEDB88320])
def test_short_hash_tables_and_merged_start(orc, poly):
    """The f4 finalize (frame_kernels.hip k_frame_finalize): lin_t equals the oracle's
    raw CRC from 0 over every (a, b) of a 32-byte window, and the derived start
    lin(seg..s) = E(ep) * x^(8 (s - bend(ep))) ^ lin(granule(ep)..s) equals
    (E(ep) * x^(-8 (bend - ep)) ^ lin(granule..ep)) * x^(8 (s - ep)) ^ lin(ep..s)."""
    rng = random.Random(poly)
    dw, b8 = _short_tables(orc, poly)
    raw = orc.crc32c_raw if poly == 0x82F63B78 else orc.crc32_raw
    base = 4096 + 16 * 7
    mem = {base + i: rng.randrange(256) for i in range(64)}
    for a in range(base, base + 16):
        for b in range(a, (a & ~15) + 33):
            want = raw(bytes(mem[x] for x in range(a, b)), 0)
            assert model_lin_t(dw, b8, mem, a, b) == want, (a - base, b - a)
    for _ in range(200):
        ep = base + rng.randrange(0, 16)
        s = ep + rng.randrange(0, 17)
        g = ep & ~15
        bend = (ep & ~1023) + 1024
        E = rng.getrandbits(32)
        old_qp = gf(orc, E, xpow_bits(orc, -8 * (bend - ep), poly), poly) ^ model_lin_t(dw, b8, mem, g, ep)
        old = gf(orc, old_qp, xpow_bits(orc, 8 * (s - ep), poly), poly) ^ model_lin_t(dw, b8, mem, ep, s)
        new = gf(orc, E, xpow_bits(orc, 8 * (s - bend), poly), poly) ^ model_lin_t(dw, b8, mem, g, s)
        assert new == old


def model_clmul32(x, y):
    """gf2.h clmul32: 16 integer products of the operands' residue classes mod 4, masked."""
    m = [0x11111111 << i for i in range(4)]
    xs, ys = [x & mi for mi in m], [y & mi for mi in m]
    z = [0] * 4
    for i in range(4):
        for j in range(4):
            z[(i + j) % 4] ^= (xs[i] * ys[j]) & 0xFFFFFFFFFFFFFFFF
    return sum(z[r] & (0x1111111111111111 << r) for r in range(4))


@pytest.mark.parametrize("poly", [0x82F63B78, 0xEDB88320])
def test_clmul_gf_mul_model(orc, poly):
    """gf2.h gf_mul_dw (the f4 finalize's multiplier): clmul32 is the carry-less product
    (checked against a bit loop), and (clmul << 1) split into its high word and the low word
    reduced by one pass through the x^32 dword tables equals the oracle's a * b mod P."""
    rng = random.Random(poly ^ 0x51)
    dw, _ = _short_tables(orc, poly)
    for _ in range(3000):
        a, b = rng.getrandbits(32), rng.getrandbits(32)
        cl = 0
        for i in range(32):
            if (b >> i) & 1:
                cl ^= a << i
        assert model_clmul32(a, b) == cl
        z = (cl << 1) & 0xFFFFFFFFFFFFFFFF
        h, lo = z >> 32, z & M32
        got = h ^ dw[0][lo & 255] ^ dw[1][(lo >> 8) & 255] ^ dw[2][(lo >> 16) & 255] ^ dw[3][lo >> 24]
        assert got == gf(orc, a, b, poly), (hex(a), hex(b))


@pytest.mark.parametrize("poly", [0x82F63B78, 0xEDB88320])
def test_lane_weight_fold_tables(orc, poly):
    """The f4 stream kernel's fold (frame_kernels.hip fold_lw / block_prefix_lw, FoldTables):
    byte tables of x^-32 (in-lane Horner), per-lane-column nibble weights x^(-128 (l % 32)) and
    byte tables of x^-4096 for lanes 32..63 give exactly sum_{l,d} s_{l,d} x^(-32 (4l + d)), and the
    half-scan + x^-4096 correction gives every exclusive lane prefix of the block."""
    rnd = random.Random(poly)

    def nib(c):  # FoldTables::w layout: [j][n] = (n << 4j) * c
        return [[gf(orc, n << (4 * j), c, poly) for n in range(16)] for j in range(8)]

    def byt(c):  # FoldTables::c0 / ch layout: [k][b] = (b << 8k) * c
        return [[gf(orc, b << (8 * k), c, poly) for b in range(256)] for k in range(4)]

    def mul_n(a, t):
        r = 0
        for j in range(8):
            r ^= t[j][(a >> (4 * j)) & 15]
        return r

    def mul_b(a, t):
        return t[0][a & 255] ^ t[1][(a >> 8) & 255] ^ t[2][(a >> 16) & 255] ^ t[3][a >> 24]

    c0, ch = byt(xpow_bits(orc, -32, poly)), byt(xpow_bits(orc, -4096, poly))
    w = [nib(xpow_bits(orc, -128 * c, poly)) for c in range(32)]
    s = [[rnd.getrandbits(32) for _ in range(4)] for _ in range(64)]
    ref = 0
    for lane in range(64):
        for d in range(4):
            ref ^= gf(orc, s[lane][d], xpow_bits(orc, -32 * (4 * lane + d), poly), poly)
    u = []  # weighted_lw per lane
    for lane in range(64):
        h = mul_b(s[lane][3], c0) ^ s[lane][2]
        h = mul_b(h, c0) ^ s[lane][1]
        h = mul_b(h, c0) ^ s[lane][0]
        u.append(mul_n(h, w[lane % 32]))
    a = b = 0
    for lane in range(32):
        a ^= u[lane]
        b ^= u[lane + 32]
    assert a ^ mul_b(b, ch) == ref  # fold_lw
    for L in range(64):  # block_prefix_lw: exclusive prefix over lanes < L
        want = 0
        for lane in range(L):
            h = mul_b(s[lane][3], c0) ^ s[lane][2]
            h = mul_b(h, c0) ^ s[lane][1]
            h = mul_b(h, c0) ^ s[lane][0]
            want ^= gf(orc, h, xpow_bits(orc, -128 * lane, poly), poly)
        x = 0
        for lane in range(32 * (L >= 32), L):
            x ^= u[lane]
        got = x if L < 32 else a ^ mul_b(x, ch)
        assert got == want, L


def test_audit_rehash_model(orc):
    """The update self-check's independent re-hash (update_kernels.hip audit_one / lin_serial,
    DESIGN.md 7): each of 64 lanes hashes its contiguous slice serially -- unaligned head and
    tail bytes through the x^8 byte table, whole dwords through the x^32 slicing tables -- the
    slices are shifted to the payload end by x^(8 (L - end)) and xor-ed, and the start term
    ~0 * x^(8 L) added.  Must equal the reference crc32c (create, Common.h:146-177) at every
    length and alignment, both polynomials."""
    rng = random.Random(77)
    for poly, ref in ((orc.POLY_CRC32C, orc.crc32c_raw), (orc.POLY_CRC32, None)):
        dw, b8 = _short_tables(orc, poly)

        def lin_serial(mem, a, b):
            c = 0
            while a < b and a % 4:
                c = (c >> 8) ^ b8[(c ^ mem[a]) & 0xFF]
                a += 1
            while a + 4 <= b:
                c ^= int.from_bytes(mem[a:a + 4], "little")
                c = dw[0][c & 0xFF] ^ dw[1][(c >> 8) & 0xFF] ^ dw[2][(c >> 16) & 0xFF] ^ dw[3][c >> 24]
                a += 4
            while a < b:
                c = (c >> 8) ^ b8[(c ^ mem[a]) & 0xFF]
                a += 1
            return c

        for L in [1, 3, 4, 5, 63, 64, 65, 255, 256, 1000, 4093, 8191]:
            base = rng.randrange(0, 16)
            mem = bytes(rng.randrange(256) for _ in range(base + L))
            slice_ = ((L + 63) // 64 + 3) & ~3
            v = 0
            for lane in range(64):
                a = min(L, lane * slice_)
                b = min(L, a + slice_)
                part = lin_serial(mem, base + a, base + b)
                if part:
                    part = gf(orc, part, xpow_bits(orc, 8 * (L - b), poly), poly)
                v ^= part
            raw = gf(orc, M32, xpow_bits(orc, 8 * L, poly), poly) ^ v
            if ref is not None:
                assert raw == ref(mem[base:base + L]), (L, base)
            else:
                import zlib
                assert raw ^ M32 == zlib.crc32(mem[base:base + L]), (L, base)


def _perm(s0, s1, sel):
    """v_perm_b32 D = perm(S0, S1, sel): byte i of D from selector byte b -- 0..3: byte b of
    S1, 4..7: byte b - 4 of S0, 0x0C: 0x00, >= 0x0D: 0xFF (the cases these kernels use)."""
    d = 0
    for i in range(4):
        b = (sel >> (8 * i)) & 0xFF
        if b < 4:
            v = (s1 >> (8 * b)) & 0xFF
        elif b < 8:
            v = (s0 >> (8 * (b - 4))) & 0xFF
        elif b == 0x0C:
            v = 0
        else:
            v = 0xFF
        d |= v << (8 * i)
    return d


def test_perm_addressed_step_tables():
    """crc_device.h (StepLds, stride_step): one v_perm_b32 per lookup address.  Table k,
    entry e, replica c at (k >> 1) * 64 KiB + e * 256 + (k & 1) * 128 + 4 c: every lane, table
    and byte value lands on its own entry of its own replica (lane l: replica l % 32, bank
    l % 32), inside the 128 KiB image."""
    rnd = random.Random(11)
    step_sel = [0x0C020400, 0x0C020501, 0x0C030600, 0x0C030701]
    for lane in range(64):
        o = (lane & 31) * 4
        c = o | ((o | 128) << 8) | (1 << 24)  # step_lds: the lane's constant
        for _ in range(64):
            x = rnd.getrandbits(32)
            for k in range(4):
                e = (x >> (8 * k)) & 0xFF
                want = (k >> 1) * 65536 + e * 256 + (k & 1) * 128 + (lane & 31) * 4
                assert _perm(x, c, step_sel[k]) == want, (lane, k, hex(x))
    assert 65536 + 255 * 256 + 128 + 31 * 4 + 4 <= 128 * 1024
