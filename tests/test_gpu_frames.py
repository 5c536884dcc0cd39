"""f4 serde frame verification, both device paths (3fs_amd/csrc/frame_kernels.h):
the stream path (sorted, disjoint frames: one pass over the receive span, the
payload CRC from two boundary values) and the per-frame record path, forced
with the library option frame_stream.  Every computed calcSerde is checked against the
oracle (Checksum::calcSerde, MessageHeader.h:33-37) and the mismatch set is
exact; layouts cover walked buffers, gaps between frames, frames spanning
many segments, empty frames at either end, unaligned buffers, unsorted
batches and oversize frames (the device falls back to the record path)."""
import os
import struct

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


@pytest.fixture(params=["1", "0"], ids=["stream", "record"])
def path(request, opts):
    opts("frame_stream", request.param)
    yield request.param


def _build(orc, rng, sizes, gaps=None, lead=0):
    """Receive buffer of serde frames (header + payload), `gaps[i]` junk bytes
    in front of frame i's header; returns (buffer, payload offsets)."""
    n = len(sizes)
    comp = rng.integers(0, 2, n)
    parts = [rng.integers(0, 256, lead, dtype=np.uint8).tobytes()]
    offs, pos = [], lead
    for i, (sz, c) in enumerate(zip(sizes, comp.tolist())):
        g = int(gaps[i]) if gaps is not None else 0
        if g:
            parts.append(rng.integers(0, 256, g, dtype=np.uint8).tobytes())
            pos += g
        payload = rng.integers(0, 256, int(sz), dtype=np.uint8).tobytes()
        parts.append(struct.pack("<II", orc.calc_serde(payload, bool(c)), int(sz)))
        parts.append(payload)
        offs.append(pos + 8)
        pos += 8 + int(sz)
    return bytearray(b"".join(parts)), offs


def _frames(L, buf, offs, sizes):
    fr = (L.Frame * len(offs))()
    for i, (o, sz) in enumerate(zip(offs, sizes)):
        ck, size = struct.unpack_from("<II", buf, o - 8)
        fr[i] = L.Frame(o, size, ck, 0, 0)
    return fr


def _corrupt(rng, buf, offs, sizes, k):
    bad = set()
    cand = [i for i, s in enumerate(sizes) if s]
    for i in rng.choice(cand, min(k, len(cand)), replace=False).tolist():
        buf[offs[i] + int(rng.integers(sizes[i]))] ^= 1 << int(rng.integers(8))
        bad.add(i)
    return bad


def _verify(L, orc, dev, buf, fr, n, max_size=1 << 20, shift=0):
    store = torch.zeros(len(buf) + 64, dtype=torch.uint8, device=dev)
    view = store[shift:shift + len(buf)]
    view.copy_(torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev))
    if isinstance(fr, list):
        fr = (L.Frame * n)(*fr)
    raw = bytes(memoryview(fr).cast("B"))
    d = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    cnt = torch.full((1,), 12345, dtype=torch.int32, device=dev)
    L.frame_verify_batch(view, d, n, max_size, cnt)
    torch.cuda.synchronize()
    out = (L.Frame * n).from_buffer_copy(d.cpu().numpy().tobytes())
    return out, int(cnt.item())


def _check(L, orc, buf, out, bad, max_size=1 << 20):
    got_bad = set()
    for i, g in enumerate(out):
        if g.size > max_size:
            assert g.status == L.INVALID_ARG, i
            got_bad.add(i)
            continue
        payload = bytes(buf[g.offset:g.offset + g.size])
        assert g.computed == orc.calc_serde(payload, bool(g.checksum & 1)), i
        if g.status:
            assert g.status == L.CHECKSUM_MISMATCH, i
            got_bad.add(i)
    return got_bad


@pytest.mark.parametrize("shift", [0, 5])
def test_frames_walked_mix(hf, orc, dev, path, shift):
    """f4's shape at 1/20 scale: the five size classes, walked, 200 corrupt."""
    L = hf._lib
    rng = np.random.default_rng(40 + shift)
    n = 50_000
    sizes = rng.choice([64, 256, 1024, 4096, 16384], n).tolist()
    buf, offs = _build(orc, rng, sizes)
    rc, frames, used = L.frame_walk(bytes(buf))
    assert rc == 0 and used == len(buf) and len(frames) == n
    bad = _corrupt(rng, buf, offs, sizes, 200)
    out, cnt = _verify(L, orc, dev, buf, frames, n, shift=shift)
    assert _check(L, orc, buf, out, bad) == bad and cnt == len(bad)


def test_frames_ragged_gaps_and_empties(hf, orc, dev, path):
    """Sizes 0..40000 (incl. 0, 1, 15, 16, 17, 1023, 1024, 1025), junk gaps
    of 0..100 bytes between frames, empty frames first and last."""
    L = hf._lib
    rng = np.random.default_rng(41)
    n = 6000
    sizes = rng.choice([0, 1, 3, 15, 16, 17, 63, 1023, 1024, 1025, 4097], n)
    sizes[::4] = rng.integers(0, 40000, sizes[::4].size)
    sizes[0] = sizes[-1] = 0
    sizes = sizes.tolist()
    gaps = rng.integers(0, 101, n)
    buf, offs = _build(orc, rng, sizes, gaps=gaps, lead=3)
    fr = _frames(L, buf, offs, sizes)
    bad = _corrupt(rng, buf, offs, sizes, 150)
    out, cnt = _verify(L, orc, dev, buf, fr, n, shift=11)
    assert _check(L, orc, buf, out, bad) == bad and cnt == len(bad)


def test_frames_spanning_many_segments(hf, orc, dev, path):
    """Few large frames: each payload spans many stream segments (the
    finalize's Horner over segment values)."""
    L = hf._lib
    rng = np.random.default_rng(42)
    sizes = [1 << 20, 700_001, 1, 0, (1 << 20) - 3, 333_333] * 50
    n = len(sizes)
    buf, offs = _build(orc, rng, sizes, gaps=rng.integers(0, 40, n))
    fr = _frames(L, buf, offs, sizes)
    bad = _corrupt(rng, buf, offs, sizes, 40)
    out, cnt = _verify(L, orc, dev, buf, fr, n, shift=3)
    assert _check(L, orc, buf, out, bad) == bad and cnt == len(bad)


def test_frames_all_empty(hf, orc, dev, path):
    L = hf._lib
    rng = np.random.default_rng(43)
    n = 1000
    sizes = [0] * n
    buf, offs = _build(orc, rng, sizes)
    fr = _frames(L, buf, offs, sizes)
    out, cnt = _verify(L, orc, dev, buf, fr, n)
    assert _check(L, orc, buf, out, set()) == set() and cnt == 0


def test_frames_unsorted_and_oversize_fall_back(hf, orc, dev):
    """Batches the stream path cannot take (unsorted, overlapping, a frame
    above max_size) take the record path on the device: same results."""
    L = hf._lib
    rng = np.random.default_rng(44)
    n = 4000
    sizes = rng.choice([10, 100, 1000, 3000, 20000], n).tolist()
    buf, offs = _build(orc, rng, sizes)
    fr = _frames(L, buf, offs, sizes)
    bad = _corrupt(rng, buf, offs, sizes, 80)
    perm = rng.permutation(n)
    shuffled = (L.Frame * n)(*[fr[int(i)] for i in perm])
    out, cnt = _verify(L, orc, dev, buf, shuffled, n)
    assert _check(L, orc, buf, out, {int(np.nonzero(perm == i)[0][0]) for i in bad}) == \
        {int(np.nonzero(perm == i)[0][0]) for i in bad} and cnt == len(bad)
    # overlapping: frame 1 re-verified as a sub-range of frame 0's payload is
    # still a valid request (its own checksum field), only the layout differs
    dup = (L.Frame * n)(*fr)
    dup[1] = L.Frame(fr[0].offset, min(fr[0].size, 5), fr[1].checksum, 0, 0)
    out, cnt = _verify(L, orc, dev, buf, dup, n)
    got = _check(L, orc, buf, out, set())
    assert bad - {1} <= got
    # one frame above max_size: kInvalidArg for it only
    out, cnt = _verify(L, orc, dev, buf, fr, n, max_size=10000)
    got = _check(L, orc, buf, out, bad, max_size=10000)
    assert got == bad | {i for i, s in enumerate(sizes) if s > 10000} and cnt == len(got)


def test_frames_sparse_stay_on_record_path(hf, orc, dev, path):
    """Sorted but sparse frames: 400 small payloads scattered over a
    40 MB receive buffer.  The stream path would read the whole span, so the
    device check sends the batch to the record path (gap bytes beyond the
    headers exceed the payload bytes); every value and the mismatch set stay
    exact, and a dense neighbour batch in the same buffer still streams."""
    L = hf._lib
    rng = np.random.default_rng(45)
    n = 400
    sizes = rng.choice([1, 64, 200, 4096], n).tolist()
    gaps = rng.integers(90_000, 110_000, n)
    buf, offs = _build(orc, rng, sizes, gaps=gaps, lead=7)
    fr = _frames(L, buf, offs, sizes)
    bad = _corrupt(rng, buf, offs, sizes, 30)
    out, cnt = _verify(L, orc, dev, buf, fr, n, shift=1)
    assert _check(L, orc, buf, out, bad) == bad and cnt == len(bad)


def test_frames_boundary_at_every_granule(hf, orc, dev, path):
    """Frame ends at every byte position of a 1 KiB block, one boundary per block (the
    stream path's sparse fold, boundary granule 0..63 and block edges) and, in the
    second half, several per block (the dense prefix path)."""
    L = hf._lib
    rng = np.random.default_rng(46)
    sparse = [2048 + d for d in range(0, 1040)]  # ends walk every offset mod 1024
    dense = rng.integers(0, 200, 3000).tolist()
    sizes = sparse + dense
    n = len(sizes)
    buf, offs = _build(orc, rng, sizes, lead=int(rng.integers(0, 16)))
    fr = _frames(L, buf, offs, sizes)
    bad = _corrupt(rng, buf, offs, sizes, 60)
    for shift in (0, 8):
        out, cnt = _verify(L, orc, dev, buf, fr, n, shift=shift)
        assert _check(L, orc, buf, out, bad) == bad and cnt == len(bad)
