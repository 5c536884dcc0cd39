"""GPU parity of the record batches on either side of the path:
stored-chunk scrub against persisted checksums (f3) and serde frame checksum
verification (f4), against the oracle, with exact mismatch sets."""
import ctypes
import random
import struct

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
M32 = 0xFFFFFFFF


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _records_to_dev(recs, dev):
    raw = b"".join(bytes(r) for r in recs)
    return torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)


def _records_from_dev(t, cls, n):
    raw = t.cpu().numpy().tobytes()
    sz = ctypes.sizeof(cls)
    return [cls.from_buffer_copy(raw[i * sz:(i + 1) * sz]) for i in range(n)]


@pytest.mark.parametrize("ctype", [1, 2])
def test_scrub_vs_oracle(hf, orc, dev, ctype):
    L = hf._lib
    rnd = random.Random(21 + ctype)
    rng = np.random.default_rng(21 + ctype)
    size = 48 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = torch.from_numpy(host).to(dev)
    n, max_len = 700, 4 << 20
    recs, want = [], []
    for i in range(n):
        ln = rnd.choice([0, 1, 3, 4096, 65536, 131072 + 7, rnd.randrange(0, 300000), max_len])
        off = rnd.randrange(0, size - ln)
        data = host[off:off + ln]
        fin = rnd.randrange(2) if ctype == 1 else 0
        typ = 0 if rnd.random() < 0.1 else ctype
        raw = orc.create(ctype, data)[1]
        stored = (~raw & M32) if fin else raw
        if rnd.random() < 0.15:  # corrupted persisted value
            stored ^= 1 << rnd.randrange(32)
        r = L.ScrubIO(data=arena.data_ptr() + off, length=ln, checksum_type=typ, fin=fin, checksum=stored)
        if rnd.random() < 0.02:  # malformed records
            if ctype == 1 and typ:
                r.checksum_type = 2
            else:
                r.fin = 7
        recs.append(r)
        if r.checksum_type not in (0, ctype) or r.fin > 1:
            want.append((L.INVALID_ARG, 0))
        else:
            want.append(orc.scrub(r.checksum_type, r.fin, data, stored))
    d = _records_to_dev(recs, dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    L.scrub_batch(ctype, d, n, max_len, cnt)
    torch.cuda.synchronize()
    got = _records_from_dev(d, L.ScrubIO, n)
    assert [(g.status, g.computed) for g in got] == want
    assert int(cnt.item()) == sum(1 for s, _ in want if s)
    assert any(s == L.CHECKSUM_MISMATCH for s, _ in want) and any(s == 0 for s, _ in want)


def test_frame_verify_vs_oracle(hf, orc, dev):
    L = hf._lib
    rnd = random.Random(8)
    buf = bytearray()
    sizes = []
    for _ in range(2500):
        size = rnd.choice([0, 1, 5, 64, 512, 4096, 65536, rnd.randrange(0, 100000)])
        payload = rnd.randbytes(size)
        comp = rnd.randrange(2)
        buf += struct.pack("<II", orc.calc_serde(payload, bool(comp)), size) + payload
        sizes.append(size)
    # corrupt some payload bytes (header left intact so the walk still frames them)
    rc, frames, used = L.frame_walk(bytes(buf))
    assert rc == 0 and used == len(buf) and len(frames) == len(sizes)
    bad = set()
    for i in rnd.sample(range(len(frames)), 60):
        f = frames[i]
        if f.size:
            buf[f.offset + rnd.randrange(f.size)] ^= 1 << rnd.randrange(8)
            bad.add(i)
    n = len(frames)
    dbuf = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
    dfr = _records_to_dev(frames, dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    L.frame_verify_batch(dbuf, dfr, n, 1 << 20, cnt)
    torch.cuda.synchronize()
    got = _records_from_dev(dfr, L.Frame, n)
    for i, g in enumerate(got):
        payload = bytes(buf[g.offset:g.offset + g.size])
        assert g.computed == orc.calc_serde(payload, bool(g.checksum & 1)), i
        assert (g.status == L.CHECKSUM_MISMATCH) == (i in bad), i
    assert int(cnt.item()) == len(bad)
    # size above max_size -> kInvalidArg for that frame only
    dfr2 = _records_to_dev(frames[:50], dev)
    L.frame_verify_batch(dbuf, dfr2, 50, 1000, cnt)
    torch.cuda.synchronize()
    got2 = _records_from_dev(dfr2, L.Frame, 50)
    for f, g in zip(frames[:50], got2):
        if f.size > 1000:
            assert g.status == L.INVALID_ARG
        else:
            assert g.status in (0, L.CHECKSUM_MISMATCH)


def test_frame_verify_many_small_frames(hf, orc, dev):
    """f4's shape: > 16 frames per wave, all <= 16 KiB, so the record job's
    device-side length bound takes the cross-task head prefetch
    (crc_kernels.hip direct_pipe); every computed calcSerde against the oracle,
    exact mismatch set."""
    L = hf._lib
    rng = np.random.default_rng(21)
    n = 80_000
    sizes = rng.choice([0, 1, 5, 64, 256, 1024, 4096, 16384], n)
    sizes[::3] = rng.integers(0, 16385, sizes[::3].size)
    comp = rng.integers(0, 2, n)
    pool = rng.integers(0, 256, int(sizes.sum()) + 16, dtype=np.uint8).tobytes()
    parts, pos = [], 0
    for sz, c in zip(sizes.tolist(), comp.tolist()):
        payload = pool[pos:pos + sz]
        pos += sz
        parts.append(struct.pack("<II", orc.calc_serde(payload, bool(c)), sz))
        parts.append(payload)
    buf = bytearray(b"".join(parts))
    rc, frames, used = L.frame_walk(bytes(buf))
    assert rc == 0 and used == len(buf) and len(frames) == n
    bad = set()
    for i in rng.choice(n, 300, replace=False).tolist():
        f = frames[i]
        if f.size:
            buf[f.offset + int(rng.integers(f.size))] ^= 1 << int(rng.integers(8))
            bad.add(i)
    dbuf = torch.frombuffer(buf, dtype=torch.uint8).to(dev)
    dfr = _records_to_dev(frames, dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    L.frame_verify_batch(dbuf, dfr, n, 1 << 20, cnt)
    torch.cuda.synchronize()
    got = _records_from_dev(dfr, L.Frame, n)
    for i, g in enumerate(got):
        assert g.computed == orc.calc_serde(bytes(buf[g.offset:g.offset + g.size]), bool(g.checksum & 1)), i
    assert {i for i, g in enumerate(got) if g.status == L.CHECKSUM_MISMATCH} == bad
    assert int(cnt.item()) == len(bad)
