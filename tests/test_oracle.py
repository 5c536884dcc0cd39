"""CPU oracle pinned against the reference's known answers and the golden vectors.

Reference pins: tests/common/utils/TestFolly.cc:11-21, the VerifyChecksum
write patterns of tests/storage/client/TestStorageClientInterface.cc:357-462,
chunk engine tests engine.rs:816-845,1259-1332, ChecksumInfo semantics
src/fbs/storage/Common.h:113-202.
"""
import hashlib
import random
import zlib

import numpy as np
import pytest

M32 = 0xFFFFFFFF


def test_known_answers(orc):
    assert (~orc.crc32c_raw(b"123456789")) & M32 == 0xE3069283  # RFC 3720
    assert (~orc.crc32c_raw(bytes(1 << 20))) & M32 == 0x14298C12  # TestFolly.cc:20
    assert (~orc.crc32c_raw(bytes(1))) & M32 == 0x527D5351  # TestFolly.cc:21
    for kind in ("hw", "sw", "clmul", "pclmul128"):
        assert orc.crc32c_raw(b"123456789", kind=kind) == 0x1CF96D7C
        assert (~orc.crc32c_raw(bytes(1 << 20), kind=kind)) & M32 == 0x14298C12  # TestFolly.cc:20


def test_clmul_leg_matches_sse42(orc, golden):
    """The carry-less folding leg (bench.py cpu_baseline's second CPU form) against the
    SSE4.2 leg and the golden vectors: every length 0..1100 (the 128 / 256 / 512-byte
    fold thresholds and every tail), random alignments, start values, and multi-MiB buffers."""
    rng = np.random.default_rng(2026)
    base = rng.integers(0, 256, (4 << 20) + 64, dtype=np.uint8)
    for n in range(0, 1101):
        off, st = int(rng.integers(0, 64)), int(rng.integers(0, 1 << 32))
        d = base[off:off + n]
        want = orc.crc32c_raw(d, st, kind="hw")
        assert orc.crc32c_raw(d, st, kind="clmul") == want, (n, off)
        assert orc.crc32c_raw(d, st, kind="pclmul128") == want, (n, off)
    for n in (4095, 4096, 65536 + 17, (1 << 20) - 1, (4 << 20) + 3):
        off = int(rng.integers(0, 64))
        d = base[off:off + n]
        assert orc.crc32c_raw(d, kind="clmul") == orc.crc32c_raw(d, kind="sw"), n
    for v in golden["synth"]:
        d = orc.fill_synth(v["len"], golden["seed"], v["chunk_id"], v["byte_off"])
        assert orc.crc32c_raw(d, kind="clmul") == v["crc32c_raw"]
    arr = rng.integers(0, 256, (16, 300 << 10), dtype=np.uint8)
    assert np.array_equal(np.asarray(orc.create_batch(arr, threads=2, kind=2)),
                          np.asarray(orc.create_batch(arr, threads=1, kind=0)))


def test_folly_combine_identity(orc):
    # TestFolly.cc:11-18: crc32c_combine(crc1, crc2, 5) == crc32c("world", 5, crc1)
    crc1 = orc.crc32c_raw(b"hello", 0)
    crc2 = orc.crc32c_raw(b"world", 0)
    assert orc.crc32c_combine(crc1, crc2, 5) == orc.crc32c_raw(b"world", crc1)
    # the logged line of TestFolly.cc:20-22: crc32c_combine(~crc32c1, crc32c2, 1) with crc32c1 =
    # ~0x14298C12 (raw CRC of 1 MiB of zeros) and crc32c2 = ~0x527D5351 (raw CRC of one zero byte)
    # is the raw CRC of the concatenation, 1 MiB + 1 zero bytes
    out = orc.crc32c_combine(0x14298C12, ~0x527D5351 & M32, 1)
    assert out == orc.crc32c_raw(bytes((1 << 20) + 1))


def test_golden_strings(orc, golden):
    for s in golden["strings"]:
        d = bytes.fromhex(s["hex"])
        assert orc.crc32c_raw(d) == s["crc32c_raw"]
        assert orc.crc32c_raw(d, kind="sw") == s["crc32c_raw"]
        assert orc.crc32c_raw(d, 0) == s["crc32c_raw_start0"]
        assert orc.crc32_raw(d) == s["crc32_raw"]
        assert (~orc.crc32_raw(d)) & M32 == zlib.crc32(d)


def test_golden_synth(orc, golden):
    for v in golden["synth"]:
        d = orc.fill_synth(v["len"], golden["seed"], v["chunk_id"], v["byte_off"])
        assert hashlib.sha256(d.tobytes()).hexdigest() == v["sha256"], v
        assert orc.crc32c_raw(d) == v["crc32c_raw"]
        assert orc.crc32c_raw(d, kind="sw") == v["crc32c_raw"]
        assert orc.crc32c_raw(d, 0) == v["crc32c_raw_start0"]
        assert orc.crc32c_raw(d, 0x12345678) == v["crc32c_raw_start_custom"]
        assert orc.crc32_raw(d) == v["crc32_raw"]
        assert orc.create(1, d) == (1, v["crc32c_raw"])
        assert orc.create(2, d) == (2, v["crc32_raw"])


def test_golden_combine(orc, golden):
    for v in golden["combine"]:
        assert orc.crc32c_combine(v["c1"], v["c2"], v["len2"]) == v["crc32c"]
        assert orc.crc32_combine(v["c1"], v["c2"], v["len2"]) == v["crc32"]


def test_hw_sw_bitwise_agree(orc):
    rng = np.random.default_rng(1)
    for n in [0, 1, 7, 8, 255, 256, 767, 768, 769, 3 * 8192 - 1, 3 * 8192, 3 * 8192 + 9, 100000]:
        d = rng.integers(0, 256, n, dtype=np.uint8)
        for off in (0, 1, 5):
            x = d[off:]
            a = orc.crc32c_raw(x, 0xDEADBEEF)
            assert a == orc.crc32c_raw(x, 0xDEADBEEF, kind="sw")
            if n < 5000:
                assert a == orc.bitwise(x, 0xDEADBEEF, orc.POLY_CRC32C)


def test_checksuminfo_semantics(orc):
    d = b"some data"
    assert orc.create(0, d) == (0, 0)  # NONE -> {NONE, 0} (Common.h:150)
    assert orc.create(1, b"") == (1, M32)  # length 0 -> {type, start}
    assert orc.create(1, b"", 0x1234) == (1, 0x1234)
    # combine: type mismatch -> kChecksumMismatch (Common.h:180-183)
    rc, _ = orc.combine((1, 5), (2, 6), 10)
    assert rc == orc.CHECKSUM_MISMATCH
    # length 0 -> no-op even for NONE (:184)
    assert orc.combine((0, 0), (1, 7), 0) == (0, (0, 0))
    assert orc.combine((1, 9), (1, 7), 0) == (0, (1, 9))
    # NONE self -> copy (:186-188)
    assert orc.combine((0, 0), (1, 7), 3) == (0, (1, 7))
    # CRC32C / CRC32 concatenation
    a, b = b"abcdefghij" * 37, b"0123456789" * 11
    for t in (1, 2):
        rc, c = orc.combine(orc.create(t, a), orc.create(t, b), len(b))
        assert rc == 0 and c == orc.create(t, a + b)


def test_calc_serde(orc):
    # MessageHeader.h:33-37: crc32c init 0, low byte = 0x86 | compressed
    d = b"serde frame payload"
    c = orc.crc32c_raw(d, 0)
    assert orc.calc_serde(d) == (c & ~0xFF & M32) | 0x86
    assert orc.calc_serde(d, True) == (c & ~0xFF & M32) | 0x87


@pytest.mark.parametrize("chunk_size", [512, 128 * 1024])
def test_replica_verify_checksum_patterns(orc, chunk_size):
    """TestStorageClientInterface.cc:357-462 VerifyChecksum: after SEQ/JUMP/RAND
    writes the chunk checksum equals crc32c(chunk bytes)."""
    rnd = random.Random(chunk_size)
    for pattern in ("SEQ", "JUMP", "RAND"):
        chunk = bytearray(chunk_size)
        size, ck = 0, (0, 0)
        offset = length = 0
        for _ in range(100):
            if pattern == "SEQ":
                offset += length
            elif pattern == "JUMP":
                offset += length + rnd.randint(0, length // 2)
            else:
                offset = rnd.randint(0, chunk_size)
            if offset + 1 >= chunk_size:
                continue
            length = rnd.randint(1, (chunk_size - offset) // 2)
            payload = bytes(rnd.getrandbits(8) for _ in range(length))
            wck = orc.create(1, payload)
            rc, size, ck = orc.replica_apply(chunk, size, ck, orc.WRITE, offset, length, payload, wck)
            assert rc == 0
            assert ck == (1, orc.crc32c_raw(bytes(chunk[:size])))


def test_replica_cases_and_truncate(orc):
    chunk = bytearray(4096)
    rng = random.Random(7)
    data = bytes(rng.getrandbits(8) for _ in range(1000))
    # first write at 0: reuse (case 2)
    rc, size, ck = orc.replica_apply(chunk, 0, (0, 0), orc.WRITE, 0, 1000, data, orc.create(1, data))
    assert (rc, size, ck) == (0, 1000, orc.create(1, data))
    # bad payload checksum -> kChecksumMismatch, nothing changes
    rc, size2, ck2 = orc.replica_apply(chunk, size, ck, orc.WRITE, 10, 10, data, (1, 123))
    assert (rc, size2, ck2) == (orc.CHECKSUM_MISMATCH, size, ck)
    # truncate shrink / extend grow / NONE write
    rc, size, ck = orc.replica_apply(chunk, size, ck, orc.TRUNCATE, 0, 600)
    assert (rc, size, ck) == (0, 600, (1, orc.crc32c_raw(bytes(chunk[:600]))))
    rc, size, ck = orc.replica_apply(chunk, size, ck, orc.EXTEND, 0, 3000)
    assert (rc, size, ck) == (0, 3000, (1, orc.crc32c_raw(bytes(chunk[:3000]))))
    assert bytes(chunk[600:3000]) == bytes(2400)
    rc, size, ck = orc.replica_apply(chunk, size, ck, orc.TRUNCATE, 0, 0)
    assert (rc, size, ck) == (0, 0, (1, 0))  # size 0 -> value 0 (ChunkReplica.cc:334-336)
    rc, size, ck = orc.replica_apply(chunk, size, ck, orc.WRITE, 5, 10, data, (0, 0))
    assert (rc, size, ck) == (0, 15, (0, 0))
    # out of chunk bounds -> kInvalidArg
    assert orc.replica_apply(chunk, size, ck, orc.WRITE, 4096, 1, data, (0, 0))[0] == orc.INVALID_ARG


def test_engine_checksum(orc):
    """engine.rs:1259-1282: "etc" then "zzz" appended; chunk crc == crc32c(buf)."""
    buf = bytearray(1 << 16)
    rc, n, ck = orc.engine_apply(buf, 0, 0, b"etc", 0, len(buf), exists=False)
    assert rc == 0 and n == 3 and ck == orc.rs_crc32c(b"etc")
    rc, n, ck = orc.engine_apply(buf, n, ck, b"zzz", 3, len(buf))
    assert rc == 0 and n == 6 and ck == orc.rs_crc32c(b"etczzz")
    assert orc.rs_combine(orc.rs_crc32c(b"etc"), orc.rs_crc32c(b"zzz"), 3) == orc.rs_crc32c(b"etczzz")
    assert orc.rs_append(orc.rs_crc32c(b"etc"), b"zzz") == orc.rs_crc32c(b"etczzz")
    # checksum mismatch (engine.rs:297-311 -> 4080 via cxx.rs:159)
    rc, _, _ = orc.engine_apply(buf, n, ck, b"abc", 6, len(buf), data_ck=1)
    assert rc == orc.CHECKSUM_MISMATCH


def test_engine_random_writes(orc):
    """engine.rs:816-845: meta checksum == crc32c(bytes) after every kind of write."""
    rnd = random.Random(3)
    cap = 64 * 1024
    buf = bytearray(cap)
    n, ck, exists = 0, 0, False
    for it in range(200):
        kind = rnd.random()
        if kind < 0.15 and n > 0:  # truncate
            off = rnd.randint(0, n)
            rc, n, ck = orc.engine_apply(buf, n, ck, b"", off, cap, truncate=True, exists=exists)
        else:
            if kind < 0.5:
                off = n  # append
            elif kind < 0.6:
                off = (n + 4095) // 4096 * 4096 + rnd.choice([0, 4096])  # aligned gap
            else:
                off = rnd.randint(0, n + 100)
            ln = rnd.choice([rnd.randint(1, 3000), 4096, 8192])
            if off + ln > cap:
                continue
            data = bytes(rnd.getrandbits(8) for _ in range(ln))
            rc, n, ck = orc.engine_apply(buf, n, ck, data, off, cap, exists=exists)
        assert rc == 0
        exists = True
        assert ck == orc.rs_crc32c(bytes(buf[:n])), it


def test_read_result_cases(orc):
    chunk = bytes(range(256)) * 10
    ck = orc.create(1, chunk)
    # NONE batch -> {NONE, 0}
    assert orc.read_result(0, ck, 0, chunk, len(chunk)) == (0, (0, 0))
    # full-chunk read reuses the stored checksum (BatchReadJob.cc:30-31)
    assert orc.read_result(1, (1, 42), 0, chunk, len(chunk)) == (0, (1, 42))
    # partial read computes (:32-35)
    assert orc.read_result(1, ck, 100, chunk[100:300], len(chunk)) == (0, orc.create(1, chunk[100:300]))
    # resync recalculation detects a stale stored checksum (:43-54)
    rc, _ = orc.read_result(1, (1, 42), 0, chunk, len(chunk), full_chunk=chunk, recalculate=True)
    assert rc == orc.CHECKSUM_MISMATCH
    rc, _ = orc.read_result(1, ck, 0, chunk, len(chunk), full_chunk=chunk, recalculate=True)
    assert rc == 0


def test_batch_baseline_matches(orc):
    a = np.stack([orc.fill_synth(70000, 5, i) for i in range(8)])
    ref = [orc.crc32c_raw(r) for r in a]
    assert list(orc.create_batch(a, threads=1, kind=0)) == ref
    assert list(orc.create_batch(a, threads=4, kind=0)) == ref
    assert list(orc.create_batch(a, threads=2, kind=1)) == ref


def test_bulk_golden_table(orc, bulk_golden):
    """The full-size table bench.py and the GPU tests compare against: file
    integrity, sampled re-derivation by the oracle (both CRC forms), chunk 0
    by the independent pure-Python CRC + generator of make_golden.py, and the
    whole-batch pin as a combine fold of the first 4096 digests."""
    import hashlib
    import os
    import sys
    meta, table = bulk_golden
    assert table.size == meta["chunks"] == 32768
    assert hashlib.sha256(table.tobytes()).hexdigest() == meta["sha256"]
    chunk, seed = meta["chunk_bytes"], meta["seed"]
    for i in (1, 4095, 4096, 20000, 32767):
        d = orc.fill_synth(chunk, seed, i)
        assert orc.crc32c_raw(d) == int(table[i])
        assert orc.crc32c_raw(d, kind="sw") == int(table[i])
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_golden as mg  # independent pure-Python CRC and splitmix64
    d0 = mg.synth(chunk, seed, 0)
    assert d0 == orc.fill_synth(chunk, seed, 0).tobytes()
    assert mg.crc_raw(d0, M32, mg.TC) == int(table[0])
    assert orc.crc32c_raw(np.frombuffer(table[:4096].tobytes(), dtype=np.uint8)) == meta["table_crc32c_raw_first_4096"]
    acc = (orc.CRC32C, int(table[0]))
    for i in range(1, 4096):
        rc, acc = orc.combine(acc, (orc.CRC32C, int(table[i])), chunk)
        assert rc == 0
    assert acc[1] == meta["whole_batch_crc32c_raw_first_4096"]
