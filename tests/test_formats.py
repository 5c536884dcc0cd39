"""Host-side formats around the checksum path (no GPU needed): the chunk
engine's persisted ChunkMeta (derse wire form + default etag)
and the serde message framing walk (f4).  Pinned by the reference's own
ChunkMeta vector (tests/golden/reference_vectors.json) and by the oracle's
Checksum::calcSerde restatement."""
import json
import os
import random
import struct

import pytest

M32 = 0xFFFFFFFF
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def refvec():
    with open(os.path.join(HERE, "golden", "reference_vectors.json")) as f:
        return json.load(f)


def test_engine_meta_reference_vector(hf, refvec):
    L = hf._lib
    v = refvec["engine_chunk_meta"]
    data = bytes(v["bytes"])
    rc, m, used = L.engine_meta_decode(data)
    assert rc == 0 and used == len(data)
    f = v["fields"]
    assert m.pos == (f["pos_group_chunk_size"] << 32) | f["pos_index"]
    assert (m.chain_ver, m.chunk_ver, m.len, m.checksum) == (f["chain_ver"], f["chunk_ver"], f["len"], f["checksum"])
    assert (m.timestamp, m.last_request_id, m.last_client_low, m.last_client_high) == (0, 0, 0, 0)
    assert bytes(m.etag[:m.etag_len]).decode() == f["etag"] and m.uncommitted == int(f["uncommitted"])
    rc, enc = L.engine_meta_encode(m)
    assert rc == 0 and enc == data


def test_engine_meta_roundtrip_and_rejects(hf):
    L = hf._lib
    rnd = random.Random(5)
    for _ in range(200):
        m = L.EngineMeta()
        m.pos = rnd.getrandbits(64)
        m.chain_ver, m.chunk_ver, m.len, m.checksum = (rnd.getrandbits(32) for _ in range(4))
        m.timestamp, m.last_request_id, m.last_client_low, m.last_client_high = (rnd.getrandbits(64) for _ in range(4))
        m.etag_len = rnd.randrange(0, 63)
        for i in range(m.etag_len):
            m.etag[i] = rnd.getrandbits(8)
        m.uncommitted = rnd.randrange(2)
        rc, enc = L.engine_meta_encode(m)
        assert rc == 0 and enc[0] == len(enc) - 1 == 58 + m.etag_len
        # fixed little-endian layout (chunk_meta.rs field order)
        assert struct.unpack_from("<QIIIIQQQQ", enc, 1) == (m.pos, m.chain_ver, m.chunk_ver, m.len, m.checksum,
                                                             m.timestamp, m.last_request_id, m.last_client_low,
                                                             m.last_client_high)
        rc, back, used = L.engine_meta_decode(enc + b"trailing")
        assert rc == 0 and used == len(enc)
        assert bytes(back) == bytes(m)
    good = L.engine_meta_encode(m)[1]
    assert L.engine_meta_decode(good[:-1])[0] == L.INVALID_ARG                    # truncated
    assert L.engine_meta_decode(bytes([good[0] + 1]) + good[1:] + b"\0")[0] == L.INVALID_ARG  # length mismatch
    assert L.engine_meta_decode(bytes([0x80]) + good[1:])[0] == L.INVALID_ARG      # multi-byte length (unpinned)
    bad = bytearray(good)
    bad[-1] = 2                                                                  # bool out of range
    assert L.engine_meta_decode(bytes(bad))[0] == L.INVALID_ARG
    assert L.engine_meta_decode(b"")[0] == L.INVALID_ARG


def test_default_etag_is_upper_hex(hf):
    """ChunkMeta::set_default_etag_if_need: format!("{:X}", checksum) (chunk_meta.rs:30-34)."""
    L = hf._lib
    rnd = random.Random(9)
    for v in [0, 1, 0xF, 0x10, 0xABCDEF, M32] + [rnd.getrandbits(32) for _ in range(300)]:
        assert L.default_etag(v) == format(v, "X")


def _frames(orc, rnd, n):
    buf = bytearray()
    exp = []
    for _ in range(n):
        size = rnd.choice([0, 1, 7, 100, 1000, 4096, rnd.randrange(0, 70000)])
        payload = bytes(rnd.getrandbits(8) for _ in range(size)) if size < 5000 else rnd.randbytes(size)
        comp = rnd.randrange(2)
        ck = orc.calc_serde(payload, bool(comp))
        buf += struct.pack("<II", ck, size) + payload
        exp.append((len(buf) - size, size, ck))
    return bytes(buf), exp


def test_frame_walk(hf, orc):
    """Processor::unpackMsg (Processor.h:85-107): complete serde frames in order."""
    L = hf._lib
    rnd = random.Random(3)
    buf, exp = _frames(orc, rnd, 40)
    rc, fr, used = L.frame_walk(buf)
    assert rc == 0 and used == len(buf)
    assert [(f.offset, f.size, f.checksum) for f in fr] == exp
    assert all((f.checksum & 0xFE) == 0x86 for f in fr)
    # incomplete payload / header: the frames before it, then kInvalidArg
    rc, fr2, used2 = L.frame_walk(buf[:-1])
    assert rc == L.INVALID_ARG and len(fr2) == len(exp) - 1 and used2 == exp[-1][0] - 8
    rc, fr3, _ = L.frame_walk(buf + b"\x86\x00\x00")
    assert rc == L.INVALID_ARG and len(fr3) == len(exp)
    # a non-serde header (low byte not 0x86/0x87) stops the walk
    bad = bytearray(buf)
    off = exp[5][0] - 8
    bad[off] = 0x11
    rc, fr4, used4 = L.frame_walk(bytes(bad))
    assert rc == L.INVALID_ARG and len(fr4) == 5 and used4 == off
    assert L.frame_walk(b"")[0] == 0
    rc, fr5, used5 = L.frame_walk(buf, max_frames=3)
    assert rc == 0 and len(fr5) == 3 and used5 == exp[2][0] + exp[2][1]


def test_calc_serde_oracle_pins(orc):
    """calcSerde = crc32c(data, init 0) with the low byte replaced (MessageHeader.h:33-37)."""
    for data in [b"", b"123456789", bytes(range(256)) * 7]:
        c = orc.crc32c_raw(data, 0)
        assert orc.calc_serde(data) == (c & ~0xFF) | 0x86
        assert orc.calc_serde(data, True) == (c & ~0xFF) | 0x87
    assert orc.crc32c_raw(b"", 0) == 0
