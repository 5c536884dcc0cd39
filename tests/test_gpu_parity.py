"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle and the golden vectors.

Bit-exact integer results are the bar.  Full-size configurations are covered
by size-independent properties (split-and-combine identity, sampled oracle
checks, corruption detection exactly on the injected set).
"""
import ctypes
import hashlib
import random

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
M32 = 0xFFFFFFFF
SEED = 0x3F5C3C00


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def u32(t):
    return t.cpu().numpy().astype(np.uint32)


def stream():
    return torch.cuda.current_stream()


def addr_tensor(addrs, dev):
    return torch.tensor(np.array(addrs, dtype=np.uint64).view(np.int64), device=dev)


def test_golden_vectors_any_alignment(hf, orc, golden, dev):
    vecs = golden["synth"]
    arena = torch.zeros(sum(v["len"] + 64 for v in vecs) + 4096, dtype=torch.uint8, device=dev)
    base = arena.data_ptr()
    addrs, lens, pos = [], [], 0
    for k, v in enumerate(vecs):
        d = orc.fill_synth(v["len"], golden["seed"], v["chunk_id"], v["byte_off"])
        assert hashlib.sha256(d.tobytes()).hexdigest() == v["sha256"]
        pos += k % 16  # every residue mod 16
        arena[pos:pos + v["len"]] = to_dev(d, dev)
        addrs.append(base + pos)
        lens.append(v["len"])
        pos += v["len"] + 64
    n = len(vecs)
    A = addr_tensor(addrs, dev)
    L = torch.tensor(lens, dtype=torch.int64, device=dev)
    mx = max(lens)
    for ctype, key in [(1, "crc32c_raw"), (2, "crc32_raw")]:
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        hf._lib.create_batch(ctype, A, L, out, n, mx, stream=stream())
        torch.cuda.synchronize()
        assert list(u32(out)) == [v[key] for v in vecs]
    for start, key in [(0, "crc32c_raw_start0"), (0x12345678, "crc32c_raw_start_custom")]:
        S = torch.tensor(np.full(n, start, dtype=np.uint32).view(np.int32), device=dev)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        hf._lib.create_batch(1, A, L, out, n, mx, starts=S, stream=stream())
        torch.cuda.synchronize()
        assert list(u32(out)) == [v[key] for v in vecs]


def test_fill_synth_matches_oracle(hf, orc, dev):
    for n_chunks, clen in [(3, 4096), (2, 1000), (5, 65536 + 8)]:
        stride = (clen + 7) // 8 * 8
        buf = torch.zeros(n_chunks * stride, dtype=torch.uint8, device=dev)
        hf._lib.fill_synth(buf, stride, clen, n_chunks, SEED, 11, stream=stream())
        torch.cuda.synchronize()
        h = buf.cpu().numpy()
        for i in range(n_chunks):
            assert np.array_equal(h[i * stride:i * stride + clen], orc.fill_synth(clen, SEED, 11 + i))


@pytest.mark.parametrize("n,length", [(1, 0), (3, 1), (7, 1023), (5, 1025), (64, 4096 * 3 + 5), (2, 4 << 20),
                                      (64, 1 << 20), (4096, 16384), (3, (4 << 20) + 13),
                                      (1024, 1 << 20), (300, (4 << 20) + 13)])
def test_create_strided(hf, orc, dev, n, length):
    """The last two cases (>= 1 GiB, not a multiple of the waves) take the byte runs placed in
    closed form (k_runs_uniform), unaligned lengths and a start value included."""
    stride = (length + 15) // 16 * 16 + 16
    buf = torch.empty(max(1, n * stride), dtype=torch.uint8, device=dev)
    hf._lib.fill_synth(buf, stride, length, n, SEED, 100, stream=stream())
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_strided(1, buf, stride, length, n, out, stream=stream())
    out2 = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_strided(2, buf, stride, length, n, out2, start=0x1111, stream=stream())
    torch.cuda.synchronize()
    h = buf.cpu().numpy()
    ref = [orc.crc32c_raw(h[i * stride:i * stride + length]) for i in range(n)]
    ref2 = [orc.crc32_raw(h[i * stride:i * stride + length], 0x1111) for i in range(n)]
    assert list(u32(out)) == ref
    assert list(u32(out2)) == ref2


def test_create_config0_exact_set(hf, orc, dev):
    """BASELINE configs[0]'s exact chunk set on the HIP path: 1024 x 512 KiB contiguous
    synthetic chunks (ids 0..1023, the bench's cpu_baseline sample), ChecksumInfo::create
    semantics (Common.h:146-177), every digest against the oracle's."""
    n, length = 1024, 512 << 10
    buf = torch.empty(n * length, dtype=torch.uint8, device=dev)
    hf._lib.fill_synth(buf, length, length, n, SEED, 0, stream=stream())
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_strided(1, buf, length, length, n, out, stream=stream())
    torch.cuda.synchronize()
    h = buf.cpu().numpy().reshape(n, length)
    assert np.array_equal(h[5], orc.fill_synth(length, SEED, 5))
    ref = np.asarray(orc.create_batch(h, threads=8), dtype=np.uint32)
    assert np.array_equal(u32(out), ref)


def test_none_type(hf, dev):
    buf = torch.ones(4096, dtype=torch.uint8, device=dev)
    out = torch.full((4,), 7, dtype=torch.int32, device=dev)
    hf._lib.create_strided(0, buf, 1024, 1024, 4, out, stream=stream())
    torch.cuda.synchronize()
    assert list(u32(out)) == [0, 0, 0, 0]  # create(NONE, ...) == {NONE, 0}


@pytest.mark.parametrize("runs", ["0", "1", "1@2", "1@5"], ids=["tasks", "byte_runs", "byte_runs_rep2", "byte_runs_rep5"])
def test_random_ranges_unaligned(hf, orc, dev, runs, opts):
    """Ragged ranges at every alignment with random start values, as segment tasks and as byte
    runs (option list_runs: the update pre hash's schedule, ranges split at exact byte shares),
    also with several runs per wave (option prehash_rep: the chip sweeps the list in windows)."""
    opts("list_runs", runs.split("@")[0])
    if "@" in runs:
        opts("prehash_rep", runs.split("@")[1])
    rng = np.random.default_rng(5)
    size = 24 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host, dev)
    n = 600
    offs = rng.integers(0, size - 300_000, n)
    lens = rng.integers(0, 300_000, n)
    lens[:20] = rng.integers(0, 40, 20)
    starts = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    A = addr_tensor([arena.data_ptr() + int(o) for o in offs], dev)
    L = torch.tensor(lens.astype(np.int64), device=dev)
    S = torch.tensor(starts.view(np.int32), device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_batch(1, A, L, out, n, int(lens.max()), starts=S, stream=stream())
    torch.cuda.synchronize()
    ref = [orc.crc32c_raw(host[o:o + l], int(s)) for o, l, s in zip(offs, lens, starts)]
    assert list(u32(out)) == ref


def test_byte_runs_ranges_past_4GiB(hf, orc, dev, opts):
    """Byte runs (option list_runs) over ranges whose byte offsets pass 2^31 and 2^32: one 4.5 GiB
    range + 3 bytes, and three ranges (1 byte, 2 GiB + 5, 17 bytes) -- each wave's start offset
    is a 64-bit word broadcast from lane 0 (a low word with bit 31 set once sign-extended over the
    high word and faulted).  Against the oracle (SSE4.2 crc32c) over the same bytes."""
    opts("list_runs", 1)
    size = (9 << 29) + 64
    d = torch.empty(size, dtype=torch.uint8, device=dev)
    hf._lib.fill_synth(d, size, size // 8 * 8, 1, SEED, 77, stream=stream())
    torch.cuda.synchronize()
    host = d.cpu().numpy()
    cases = [[(5, (9 << 29) + 3)], [(0, 1), (100, (2 << 30) + 5), ((2 << 30) + 200, 17)]]
    for ranges in cases:
        A = addr_tensor([d.data_ptr() + o for o, _ in ranges], dev)
        Ls = torch.tensor([ln for _, ln in ranges], dtype=torch.int64, device=dev)
        out = torch.zeros(len(ranges), dtype=torch.int32, device=dev)
        hf._lib.create_batch(1, A, Ls, out, len(ranges), max(ln for _, ln in ranges), stream=stream())
        torch.cuda.synchronize()
        assert list(u32(out)) == [orc.crc32c_raw(host[o:o + ln]) for o, ln in ranges]
    del d


@pytest.mark.parametrize("ctype", [1, 2], ids=["crc32c", "crc32"])
def test_range_stream_ragged_vs_oracle(hf, orc, dev, ctype, opts):
    """Option range_stream (k_crc_range_stream: a wave's byte-balanced run of whole-range
    tasks as one block stream, folds at task ends while the next task's blocks are in
    flight) on 120 k ranges: lengths 0..70 KiB at every alignment, lengths < 4, ranges whose
    start falls in the last 3 bytes of their first block (start term added explicitly),
    empty ranges mid-run, random start values; then KV blocks (verify_blocks, > 16 per wave)
    with an exact mismatch set.  Against the oracle."""
    opts("range_stream", 1)
    rng = np.random.default_rng(700 + ctype)
    size = 48 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host, dev)
    n = 120_000
    lens = rng.integers(0, 70_001, n)
    lens[::7] = rng.integers(0, 4, lens[::7].size)
    lens[3::11] = 1024 * rng.integers(1, 9, lens[3::11].size) + rng.integers(1, 4, lens[3::11].size)
    lens[5::13] = 0
    offs = rng.integers(0, size - 70_001, n)
    offs[3::11] = (offs[3::11] // 16) * 16 + 16 - (lens[3::11] % 16)  # ends on a granule: spill cases
    starts = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    A = addr_tensor([arena.data_ptr() + int(o) for o in offs], dev)
    Ls = torch.tensor(lens.astype(np.int64), device=dev)
    S = torch.tensor(starts.view(np.int32), device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_batch(ctype, A, Ls, out, n, int(lens.max()), starts=S, stream=stream())
    torch.cuda.synchronize()
    got = u32(out)
    if ctype == 1:
        ref = [orc.crc32c_raw(host[o:o + l], int(st)) for o, l, st in zip(offs, lens, starts)]
    else:
        ref = [orc.crc32_raw(host[o:o + l], int(st)) for o, l, st in zip(offs, lens, starts)]
    bad = [i for i in range(n) if int(got[i]) != ref[i]]
    assert not bad, (len(bad), bad[:5], [(int(offs[i]), int(lens[i])) for i in bad[:5]])
    # KV blocks, the d5 shape
    m = 100_000
    kl = rng.choice([4096, 8192, 16384, 32768, 65536], m).astype(np.uint32)
    ko = (rng.integers(0, (size - 65536) // 4096, m) * 4096).astype(np.uint64)
    exp = np.array([orc.crc32c_raw(host[int(o):int(o) + int(l)]) for o, l in zip(ko, kl)], dtype=np.uint32)
    flip = np.sort(rng.choice(m, 23, replace=False))
    exp[flip] ^= np.uint32(1) << rng.integers(0, 32, flip.size).astype(np.uint32)
    mism = torch.zeros(m, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    comp = torch.zeros(m, dtype=torch.int32, device=dev)
    hf._lib.verify_blocks(1, arena, torch.tensor(ko.view(np.int64), device=dev),
                          torch.tensor(kl.view(np.int32), device=dev), torch.tensor(exp.view(np.int32), device=dev),
                          mism, cnt, m, 65536, computed=comp, stream=stream())
    torch.cuda.synchronize()
    assert int(cnt.item()) == flip.size
    assert np.array_equal(np.nonzero(mism.cpu().numpy())[0], flip)


@pytest.mark.parametrize("pipe", ["1", "0"])
def test_many_small_ranges_static_stride(hf, orc, dev, pipe, opts):
    """> 16 whole-buffer tasks per wave (static stride): with option pipe = 1 each
    wave carries the next range's head loads across the fold (crc_kernels.hip
    direct_pipe); lengths 0..9000 cover ranges inside one block, inside the
    prefetched head, and past it, every 5th range is 16..40 KiB (not prefetched),
    at every alignment, with random start values."""
    opts("pipe", pipe)
    rng = np.random.default_rng(11)
    size = 32 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host, dev)
    n = 150_000
    lens = rng.integers(0, 9001, n)
    lens[::97] = rng.integers(0, 8, lens[::97].size)
    lens[1::5] = rng.integers(16 << 10, 40001, lens[1::5].size)  # past the prefetch bound: hash_grid alone
    offs = rng.integers(0, size - 40001, n)
    starts = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    A = addr_tensor([arena.data_ptr() + int(o) for o in offs], dev)
    L = torch.tensor(lens.astype(np.int64), device=dev)
    S = torch.tensor(starts.view(np.int32), device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_batch(1, A, L, out, n, int(lens.max()), starts=S, stream=stream())
    torch.cuda.synchronize()
    ref = [orc.crc32c_raw(host[o:o + l], int(s)) for o, l, s in zip(offs, lens, starts)]
    assert list(u32(out)) == ref
    out = torch.zeros(n, dtype=torch.int32, device=dev)  # CRC32 (IEEE) tables through the same loop
    hf._lib.create_batch(2, A, L, out, n, int(lens.max()), starts=S, stream=stream())
    torch.cuda.synchronize()
    ref = [orc.crc32_raw(host[o:o + l], int(s)) for o, l, s in zip(offs, lens, starts)]
    assert list(u32(out)) == ref


def test_byte_balanced_assignment_skewed(hf, orc, dev):
    """More than 16 whole-range tasks per wave, too long for the cross-task
    prefetch: each wave takes a contiguous, byte-balanced run of tasks
    (k_bal_sums / k_bal_assign in crc_kernels.hip).  Skewed on purpose: 85 % of
    the ranges empty, runs of 64 KiB ranges, a 1 MiB range, empty ranges at the
    ends, so several wave boundaries fall on one task and some waves get none."""
    rng = np.random.default_rng(23)
    size = 48 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host, dev)
    n = 90_000
    lens = np.zeros(n, dtype=np.int64)
    live = rng.random(n) < 0.15
    lens[live] = rng.integers(1, 40001, int(live.sum()))
    lens[30000:30400] = 65536
    lens[50000] = 1 << 20
    lens[:50] = 0
    lens[-50:] = 0
    offs = rng.integers(0, size - (1 << 20) - 1, n)
    A = addr_tensor([arena.data_ptr() + int(o) for o in offs], dev)
    L = torch.tensor(lens, device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_batch(1, A, L, out, n, int(lens.max()), stream=stream())
    torch.cuda.synchronize()
    ref = [orc.crc32c_raw(host[o:o + l]) for o, l in zip(offs, lens)]
    assert list(u32(out)) == ref


@pytest.mark.parametrize("n", [1, 3, 40])
def test_single_task_every_alignment(hf, orc, dev, n):
    """Small batches whose buffers all fit one task (the end-aligned grid with
    the start xor-ed into the first data bytes): every residue mod 16 and the
    lengths that put the start bytes at the very end of block 0."""
    rng = np.random.default_rng(17 + n)
    size = 4 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host, dev)
    lens_pool = [1, 3, 4, 5, 15, 16, 17, 1020, 1021, 1023, 1024, 1025, 1027, 2047, 4096, 8189, 65535, 65536]
    cases = [(a, ln) for a in range(16) for ln in lens_pool]
    for k in range(0, len(cases), n):
        chunk = cases[k:k + n]
        offs = [4096 * (j + 1) + a for j, (a, _) in enumerate(chunk)]
        lens = [ln for _, ln in chunk]
        starts = rng.integers(0, 1 << 32, len(chunk), dtype=np.uint64).astype(np.uint32)
        starts[0] = M32
        m = len(chunk)
        A = addr_tensor([arena.data_ptr() + o for o in offs], dev)
        Ln = torch.tensor(lens, dtype=torch.int64, device=dev)
        S = torch.tensor(starts.view(np.int32), device=dev)
        out = torch.zeros(m, dtype=torch.int32, device=dev)
        hf._lib.create_batch(1, A, Ln, out, m, max(lens), starts=S, stream=stream())
        torch.cuda.synchronize()
        ref = [orc.crc32c_raw(host[o:o + ln], int(s)) for o, ln, s in zip(offs, lens, starts)]
        assert list(u32(out)) == ref, chunk


def test_verify_detects_exactly_injected(hf, orc, dev):
    n, length = 256, 65536 + 100
    stride = length + 28
    buf = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    hf._lib.fill_synth(buf, stride, length, n, SEED, 0, stream=stream())
    exp = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_strided(1, buf, stride, length, n, exp, stream=stream())
    torch.cuda.synchronize()
    bad = sorted(random.Random(1).sample(range(n), 13))
    for i in bad:  # single bit flips at random positions
        p = i * stride + random.Random(i).randrange(length)
        buf[p] ^= 1 << (i % 8)
    mism = torch.zeros(n, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    hf._lib.verify_strided(1, buf, stride, length, n, exp, mism, cnt, stream=stream())
    torch.cuda.synchronize()
    assert int(cnt.item()) == len(bad)
    assert list(np.nonzero(mism.cpu().numpy())[0]) == bad
    # batch form with explicit computed output
    A = addr_tensor([buf.data_ptr() + i * stride for i in range(n)], dev)
    L = torch.full((n,), length, dtype=torch.int64, device=dev)
    comp = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.verify_batch(1, A, L, exp, mism, cnt, n, length, computed=comp, stream=stream())
    torch.cuda.synchronize()
    assert int(cnt.item()) == len(bad)
    h = buf.cpu().numpy()
    assert list(u32(comp)) == [orc.crc32c_raw(h[i * stride:i * stride + length]) for i in range(n)]


@pytest.mark.parametrize("where", ["own_streams", "null_stream"])
def test_verify_concurrent_streams_library_scratch(hf, dev, where):
    """Worker threads verifying with d_computed = NULL (the library's scratch)
    never see each other's values, whether each has its own stream or all share
    the null stream (their create / compare launches interleave there, so the
    scratch and the ticket counters are per calling thread): each thread's
    mismatch set is exactly its own injected set (SURVEY.md §8b threading:
    32 UpdateWorker / AioReadWorker threads call concurrently)."""
    import threading
    threads, iters, n, length = 8, 12, 512, 16384
    stride = length + 16
    bufs, exps, bads = [], [], []
    for k in range(threads):
        buf = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        hf._lib.fill_synth(buf, stride, length, n, SEED, 1000 * k, stream=stream())
        exp = torch.zeros(n, dtype=torch.int32, device=dev)
        hf._lib.create_strided(1, buf, stride, length, n, exp, stream=stream())
        torch.cuda.synchronize()
        bad = sorted(random.Random(100 + k).sample(range(n), 3 + k))
        for i in bad:
            buf[i * stride + (i * 7919) % length] ^= 0x10
        bufs.append(buf)
        exps.append(exp)
        bads.append(bad)
    torch.cuda.synchronize()
    errors = []

    def worker(k):
        try:
            s = torch.cuda.Stream(dev) if where == "own_streams" else None
            # the first call grows this thread's scratch; the others reuse it
            for it in range(iters):
                m = n - (it % 3)  # varying n on the same stream
                mism = torch.zeros(n, dtype=torch.uint8, device=dev)
                cnt = torch.zeros(1, dtype=torch.int32, device=dev)
                torch.cuda.synchronize()  # the tensors' fills are done before the null-stream launches
                hf._lib.verify_strided(1, bufs[k], stride, length, m, exps[k], mism, cnt, stream=s)
                if s is None:
                    torch.cuda.synchronize()
                else:
                    s.synchronize()
                want = [i for i in bads[k] if i < m]
                got = list(np.nonzero(mism[:m].cpu().numpy())[0])
                if got != want or int(cnt.item()) != len(want):
                    errors.append((k, it, got, want))
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:3]


def test_verify_blocks_kv(hf, orc, dev):
    rng = np.random.default_rng(9)
    size = 16 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host, dev)
    n = 3000
    lens = rng.choice([4096, 8192, 16384, 32768, 65536], n).astype(np.uint32)
    offs = (rng.integers(0, (size - 65536) // 4096, n) * 4096).astype(np.uint64)
    exp = np.array([orc.crc32c_raw(host[int(o):int(o) + int(l)]) for o, l in zip(offs, lens)], dtype=np.uint32)
    bad = set(rng.choice(n, 7, replace=False).tolist())
    for i in bad:
        exp[i] ^= 1 << int(rng.integers(0, 32))
    O = torch.tensor(offs.view(np.int64), device=dev)
    Ls = torch.tensor(lens.view(np.int32), device=dev)
    E = torch.tensor(exp.view(np.int32), device=dev)
    mism = torch.zeros(n, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    comp = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.verify_blocks(1, arena, O, Ls, E, mism, cnt, n, 65536, computed=comp, stream=stream())
    torch.cuda.synchronize()
    assert int(cnt.item()) == len(bad)
    assert set(np.nonzero(mism.cpu().numpy())[0].tolist()) == bad


def test_combine_batch(hf, orc, golden, dev):
    vs = golden["combine"]
    rng = np.random.default_rng(2)
    c1 = [v["c1"] for v in vs] + rng.integers(0, 1 << 32, 500, dtype=np.uint64).tolist()
    c2 = [v["c2"] for v in vs] + rng.integers(0, 1 << 32, 500, dtype=np.uint64).tolist()
    ln = [v["len2"] for v in vs] + rng.integers(0, 1 << 34, 500, dtype=np.uint64).tolist()
    n = len(c1)
    for ctype, poly in [(1, orc.POLY_CRC32C), (2, orc.POLY_CRC32)]:
        acc = torch.tensor(np.array(c1, dtype=np.uint32).view(np.int32), device=dev)
        C2 = torch.tensor(np.array(c2, dtype=np.uint32).view(np.int32), device=dev)
        L2 = torch.tensor(np.array(ln, dtype=np.uint64).view(np.int64), device=dev)
        hf._lib.combine_batch(ctype, acc, C2, L2, n, stream=stream())
        torch.cuda.synchronize()
        ref = [c1[i] if ln[i] == 0 else orc.shift(~c1[i] & M32, ln[i], poly) ^ c2[i] for i in range(n)]
        assert list(u32(acc)) == ref


@pytest.mark.parametrize("ctype", [1, 2])
def test_combine_batch_large_vs_c_oracle(hf, orc, dev, ctype):
    """k_combine's carry-less products at scale: 1 M random (acc, crc2, len2) triples, lengths up
    to 2^44 (six byte digits: the x^(2^k) tail too) and 1 in 64 zero, against the oracle's C
    combine (crc_oracle.c orc_combine_batch), both polynomials."""
    rng = np.random.default_rng(30 + ctype)
    n = 1 << 20
    acc = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    crc2 = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    len2 = rng.integers(0, 1 << 44, n, dtype=np.uint64)
    len2[::64] = 0
    len2[1::4096] = rng.integers(1 << 61, (1 << 64) - 1, len2[1::4096].size, dtype=np.uint64)  # bit count > 2^64
    d_acc = torch.from_numpy(acc.view(np.int32).copy()).to(dev)
    hf._lib.combine_batch(ctype, d_acc, torch.from_numpy(crc2.view(np.int32).copy()).to(dev),
                          torch.from_numpy(len2.view(np.int64).copy()).to(dev), n, stream=stream())
    torch.cuda.synchronize()
    ref = orc.combine_batch(acc, crc2, len2, poly=orc.POLY_CRC32C if ctype == 1 else orc.POLY_CRC32, threads=8)
    assert np.array_equal(d_acc.cpu().numpy().view(np.uint32), ref)


def test_create_host_matches(hf, orc):
    rng = np.random.default_rng(4)
    bufs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in [0, 1, 5, 4096, 100_000, 1 << 20]]
    bufs.append(rng.integers(0, 256, (40 << 20) + 3, dtype=np.uint8).tobytes())  # > one 32 MiB stage
    vals = hf._lib.create_host(1, bufs)
    assert vals == [orc.crc32c_raw(b) for b in bufs]
    vals = hf._lib.create_host(2, bufs[:4], starts=[0, 1, 2, 3])
    assert vals == [orc.crc32_raw(b, s) for b, s in zip(bufs[:4], [0, 1, 2, 3])]
    ci = hf.ChecksumInfo.create(hf.ChecksumType.CRC32C, b"123456789")
    assert str(ci) == "CRC32C#E3069283"


def test_bulk_full_size_properties(hf, orc, dev):
    """BASELINE config 2 shape (4 MiB chunks) at 1 GiB: sampled oracle parity and
    the concat identity raw(A||B) = combine(raw(A), raw_0(B)) for every chunk."""
    n, length = 256, 4 << 20
    buf = torch.empty(n * length, dtype=torch.uint8, device=dev)
    hf._lib.fill_synth(buf, length, length, n, SEED, 0, stream=stream())
    full = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_strided(1, buf, length, length, n, full, stream=stream())
    half = length // 2 + 7
    base = buf.data_ptr()
    A = addr_tensor([base + i * length for i in range(n)], dev)
    B = addr_tensor([base + i * length + half for i in range(n)], dev)
    La = torch.full((n,), half, dtype=torch.int64, device=dev)
    Lb = torch.full((n,), length - half, dtype=torch.int64, device=dev)
    ra = torch.zeros(n, dtype=torch.int32, device=dev)
    rb = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_batch(1, A, La, ra, n, half, stream=stream())
    hf._lib.create_batch(1, B, Lb, rb, n, length - half, stream=stream())
    hf._lib.combine_batch(1, ra, rb, Lb, n, stream=stream())
    torch.cuda.synchronize()
    assert torch.equal(ra, full)
    for i in random.Random(0).sample(range(n), 6):
        h = buf[i * length:(i + 1) * length].cpu().numpy()
        assert np.array_equal(h[:4096], orc.fill_synth(4096, SEED, i))
        assert int(u32(full[i:i + 1])[0]) == orc.crc32c_raw(h)


def test_bulk_bench_config_full_table(hf, bulk_golden, dev):
    """bench.py's exact workload (BASELINE configs[1]: 4096 x 4 MiB = 16 GiB,
    HBM-resident), every digest bit-exact against the oracle's full table
    (tests/golden/make_bulk_golden.py), through three kernel paths: the
    strided whole-buffer launch bench.py times, the descriptor-list path in
    1 MiB segments (the planner's choice), and the whole 16 GiB as ONE buffer (segmented + atomic
    stitching) against the combine fold of the table.  Also the chunk ids of
    rank 7 of an 8-GPU run (ids 28672..32767) on 256 chunks."""
    meta, table = bulk_golden
    n, length = 4096, meta["chunk_bytes"]
    buf = torch.empty(n * length, dtype=torch.uint8, device=dev)
    hf._lib.fill_synth(buf, length, length, n, meta["seed"], 0, stream=stream())
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_strided(1, buf, length, length, n, out, stream=stream())
    base = buf.data_ptr()
    addrs = addr_tensor([base + i * length for i in range(n)], dev)
    lens = torch.full((n,), length, dtype=torch.int64, device=dev)
    out_list = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_batch(1, addrs, lens, out_list, n, length, stream=stream())  # planner: 1 MiB segments
    one = torch.zeros(1, dtype=torch.int32, device=dev)
    hf._lib.create_strided(1, buf, n * length, n * length, 1, one, stream=stream())
    torch.cuda.synchronize()
    assert np.array_equal(u32(out), table[:n])
    assert np.array_equal(u32(out_list), table[:n])
    assert int(u32(one)[0]) == meta["whole_batch_crc32c_raw_first_4096"]
    tbl = u32(out).astype("<u4").tobytes()
    assert hashlib.sha256(tbl).hexdigest() == hashlib.sha256(table[:n].tobytes()).hexdigest()
    m, first = 256, 7 * 4096
    hf._lib.fill_synth(buf, length, length, m, meta["seed"], first, stream=stream())
    hf._lib.create_strided(1, buf, length, length, m, out, stream=stream())
    torch.cuda.synchronize()
    assert np.array_equal(u32(out[:m]), table[first:first + m])
    del buf
    torch.cuda.empty_cache()


def test_d4_full_config_windowed_runs(hf, dev):
    """BASELINE configs[3]'s full HBM-resident batch on one GPU: 1024 x 64 MiB (64 GiB) through
    create_strided, which hashes it as byte runs in four 16 GiB windows (run_rep = 4: 16 MiB per
    wave); all 1024 digests against the oracle's table.  The same bytes as
    4096 x 16 MiB whole buffers (also windowed) fold back to the 64 MiB digests through
    ChecksumInfo::combine's algebra."""
    import json
    import os
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(gdir, "bulk_64MiB_digests.json")))
    table = np.fromfile(os.path.join(gdir, "bulk_64MiB_digests.bin"), dtype="<u4")
    cs, n = meta["chunk_bytes"], meta["chunks"]
    buf = torch.empty(n * cs, dtype=torch.uint8, device=dev)
    hf._lib.fill_synth(buf, cs, cs, n, meta["seed"], 0, stream=stream())
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.create_strided(1, buf, cs, cs, n, out, stream=stream())
    q = cs // 4
    out16 = torch.zeros(4 * n, dtype=torch.int32, device=dev)
    hf._lib.create_strided(1, buf, q, q, 4 * n, out16, stream=stream())
    torch.cuda.synchronize()
    assert np.array_equal(u32(out), table[:n])
    parts = u32(out16)
    full = ~0 & 0xFFFFFFFF
    start_term = hf._lib.shift(1, full, q)  # raw(B, 0) = raw(B, ~0) ^ ~0 x^(8|B|)
    for i in list(range(0, n, 97)) + [n - 1]:
        v = int(parts[4 * i])
        for j in range(1, 4):
            v = hf._lib.crc32c_combine(v, int(parts[4 * i + j]), q) ^ start_term
        assert v == int(table[i]), i
    del buf


def test_d4_64MiB_three_sources(hf, dev):
    """BASELINE configs[3] at its chunk size: 64 MiB chunks hashed (1) HBM-resident
    (create_strided over 64 chunks = 4 GiB, and rank 7's shard of an 8-GPU node:
    chain ids 896..959), (2) from plain host memory through the library's pinned
    staging ring (hf3fs_crc_create_host, two streams), (3) in place from
    registered host memory (hf3fs_crc_host_register, zero-copy over PCIe); every
    digest against the oracle's table tests/golden/bulk_64MiB_digests.bin."""
    import importlib
    import json
    import os
    node = importlib.import_module("3fs_amd.node")
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(gdir, "bulk_64MiB_digests.json")))
    table = np.fromfile(os.path.join(gdir, "bulk_64MiB_digests.bin"), dtype="<u4")
    cs, n = meta["chunk_bytes"], 64
    buf = torch.empty(n * cs, dtype=torch.uint8, device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.fill_synth(buf, cs, cs, n, meta["seed"], 0, stream=stream())
    hf._lib.create_strided(1, buf, cs, cs, n, out, stream=stream())
    torch.cuda.synchronize()
    assert np.array_equal(u32(out), table[:n])
    ids = node.shard_chunk_ids(meta["chunks"], 7, 8)  # rank 7 of 8: chains [896, 1024)
    assert ids[0] == 896 and ids.size == meta["chunks_per_gpu"]
    hf._lib.fill_synth(buf, cs, cs, n, meta["seed"], int(ids[0]), stream=stream())
    hf._lib.create_strided(1, buf, cs, cs, n, out, stream=stream())
    torch.cuda.synchronize()
    assert np.array_equal(u32(out), table[896:896 + n])
    # host sources: 8 chunks (ids 896..903) copied out of HBM
    m = 8
    host = buf[:m * cs].cpu().numpy()
    got = hf._lib.create_host(1, [host[i * cs:(i + 1) * cs] for i in range(m)])
    assert got == [int(x) for x in table[896:896 + m]]
    del buf
    torch.cuda.empty_cache()
    reg = np.empty(m * cs, dtype=np.uint8)  # plain host memory, registered (page-locked + mapped) in place
    reg[:] = host
    d_ptr = hf._lib.host_register(reg.ctypes.data, m * cs)
    try:
        zc = torch.zeros(m, dtype=torch.int32, device=dev)
        hf._lib.create_strided(1, d_ptr, cs, cs, m, zc, stream=stream())
        torch.cuda.synchronize()
        assert np.array_equal(u32(zc), table[896:896 + m])
    finally:
        hf._lib.host_unregister(reg.ctypes.data)


def test_d5_graph_captured_verify(hf, orc, dev):
    """BASELINE configs[4] call shape: KV blocks of {4..64} KiB at 4 KiB-aligned
    arena offsets, verify_blocks captured into a hipGraph (torch.cuda.graph on a
    side stream, d_computed given, launched once outside the capture first) and
    replayed; the mismatch set equals the injected set exactly and every
    recomputed value equals the oracle's (StorageClientImpl.cc:1720-1737)."""
    rng = np.random.default_rng(44)
    size = 96 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host, dev)
    n = 80000  # > 16 per wave: the captured launch takes byte-balanced task ranges (bal slab region)
    lens = rng.choice([4096, 8192, 16384, 32768, 65536], n).astype(np.uint32)
    offs = (rng.integers(0, (size - 65536) // 4096, n) * 4096).astype(np.uint64)
    want = np.array([orc.crc32c_raw(host[int(o):int(o) + int(ln)]) for o, ln in zip(offs, lens)], dtype=np.uint32)
    exp = want.copy()
    bad = np.sort(rng.choice(n, 29, replace=False))
    exp[bad] ^= np.uint32(1) << rng.integers(0, 32, bad.size).astype(np.uint32)
    O = torch.tensor(offs.view(np.int64), device=dev)
    Ls = torch.tensor(lens.view(np.int32), device=dev)
    E = torch.tensor(exp.view(np.int32), device=dev)
    mism = torch.zeros(n, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    comp = torch.zeros(n, dtype=torch.int32, device=dev)
    cs = torch.cuda.Stream(dev)
    with torch.cuda.stream(cs):  # warm: table build, ticket slabs, first launch
        hf._lib.verify_blocks(1, arena, O, Ls, E, mism, cnt, n, 65536, computed=comp, stream=cs)
    cs.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cs):
        hf._lib.verify_blocks(1, arena, O, Ls, E, mism, cnt, n, 65536, computed=comp, stream=cs)
    for _ in range(3):
        mism.fill_(7)
        comp.zero_()
        cnt.fill_(-1)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert int(cnt.item()) == bad.size
        assert np.array_equal(np.nonzero(mism.cpu().numpy())[0], bad)
        assert np.array_equal(u32(comp), want)


def test_captured_verify_scratch_owned_by_graph(hf, orc, dev):
    """verify_blocks with d_computed = NULL captured into two graphs (no warm-up of the
    capture stream's pair buffer sizes): each captured call's verify values, ticket
    counter and balance region are buffers of its graph, so release_stream and a larger
    eager call on the same (stream, thread) pair -- which free and regrow the pair's
    buffer -- leave every replay exact.  Destroying one graph (torch already destroyed the
    hipGraph after instantiation: only the executable graph holds the reference) frees
    that graph's buffers at the next uncaptured call and leaves the other graph exact."""
    L = hf._lib
    L.release_graph_scratch()
    base = L.graph_scratch_stats()
    rng = np.random.default_rng(77)
    size = 64 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = to_dev(host, dev)
    n = 80000  # > 16 tasks per wave: the launch takes a balance region too
    lens = rng.choice([4096, 8192, 16384, 65536], n).astype(np.uint32)
    offs = (rng.integers(0, (size - 65536) // 4096, n) * 4096).astype(np.uint64)
    want = np.array([orc.crc32c_raw(host[int(o):int(o) + int(ln)]) for o, ln in zip(offs, lens)], dtype=np.uint32)
    O = torch.tensor(offs.view(np.int64), device=dev)
    Ls = torch.tensor(lens.view(np.int32), device=dev)
    cs = torch.cuda.Stream(dev)
    graphs = []
    for k in range(2):
        exp = want.copy()
        bad = np.sort(rng.choice(n, 11 + k, replace=False))
        exp[bad] ^= np.uint32(1 << (3 + k))
        E = torch.tensor(exp.view(np.int32), device=dev)
        mism = torch.zeros(n, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cs):
            L.verify_blocks(1, arena, O, Ls, E, mism, cnt, n, 65536, computed=None, stream=cs)
        graphs.append((g, bad, mism, cnt, E))
    torch.cuda.synchronize()
    owned = L.graph_scratch_stats()
    assert owned["live"] >= base["live"] + 2, (base, owned)  # the verify values (+ counter, balance) per graph
    assert owned["live_bytes"] >= base["live_bytes"] + 2 * 4 * n

    def replay_exact(g, bad, mism, cnt, E):
        mism.fill_(7)
        cnt.fill_(-1)
        g.replay()
        torch.cuda.synchronize()
        assert int(cnt.item()) == bad.size
        assert np.array_equal(np.nonzero(mism.cpu().numpy())[0], bad)

    for rec in graphs:
        replay_exact(*rec)
    L.release_stream(cs)  # frees the (cs, thread) pair's buffers
    bigger = 2 * n  # an eager call larger than any before: the pair buffer grows
    O2, L2 = O.repeat(2), Ls.repeat(2)
    E2 = torch.tensor(np.tile(want, 2).view(np.int32), device=dev)
    m2 = torch.zeros(bigger, dtype=torch.uint8, device=dev)
    c2 = torch.zeros(1, dtype=torch.int32, device=dev)
    with torch.cuda.stream(cs):
        L.verify_blocks(1, arena, O2, L2, E2, m2, c2, bigger, 65536, computed=None, stream=cs)
    cs.synchronize()
    assert int(c2.item()) == 0
    for _ in range(2):
        for rec in graphs:
            replay_exact(*rec)
    g0 = graphs.pop(0)
    del g0
    torch.cuda.synchronize()
    gone = L.graph_scratch_stats()
    assert gone["live"] < owned["live"] and gone["dead"] >= 1, (owned, gone)
    with torch.cuda.stream(cs):  # an uncaptured call below 64 MiB of dead buffers frees nothing
        L.verify_blocks(1, arena, O2, L2, E2, m2, c2, bigger, 65536, computed=None, stream=cs)
    cs.synchronize()
    assert L.graph_scratch_stats()["dead"] == gone["dead"]
    L.release_graph_scratch()  # frees the dead graph's buffers
    assert L.graph_scratch_stats()["dead"] == 0
    replay_exact(*graphs[0])
    del g, rec  # the loop variables hold the last graph too
    graphs.clear()
    torch.cuda.synchronize()
    L.release_graph_scratch()
    end = L.graph_scratch_stats()
    assert end["live"] <= base["live"] and end["dead"] == 0, (base, end)


# ---- ChunkReplica::update on device -------------------------------------------------
def _random_ios(rng, n_chunks, chunk_size, sizes, cks, pattern):
    ios = []
    for c in range(n_chunks):
        size = sizes[c]
        r = rng.random()
        if pattern == "mixed" and r < 0.08:
            ios.append(("T", rng.integers(0, chunk_size + 1)))
        elif pattern == "mixed" and r < 0.12:
            ios.append(("E", rng.integers(0, chunk_size + 1)))
        else:
            if pattern == "seq" or r < 0.3:
                off = size
            else:
                off = int(rng.integers(0, chunk_size))
            if off >= chunk_size:
                off = int(rng.integers(0, chunk_size))
            ln = int(rng.integers(1, chunk_size - off + 1))
            ln = min(ln, max(1, int(rng.integers(1, chunk_size // 2 + 2))))
            ios.append(("W", off, ln))
    return ios


def _set_pipeline(opts, pipeline):
    """"unfused": prep -> k_crc_ranges(pre) -> apply (the default apply: ticketed tasks on a
    (stream, thread) pair's first call, one-shot pieces after it); "fused": k_update_fused;
    "unfused_fine": the ticketed apply cut into up to 65 pieces of >= 1 KiB per range (the
    16-byte aligned cuts of k_update_apply land inside every write and gap);
    "oneshot_loop": the one-shot apply with 4 KiB pieces on a 256-workgroup grid (every
    workgroup loops over many pieces); "oneshot16": one-shot, 16 KiB pieces, on every call."""
    base = {"unfused_fine": "unfused", "oneshot_loop": "unfused", "oneshot16": "unfused"}
    opts("update_pipeline", base.get(pipeline, pipeline))
    if pipeline == "unfused_fine":
        opts("apply_grid", 0)
        opts("apply_pieces", 64)
        opts("apply_min_kib", 1)
    if pipeline == "oneshot_loop":
        opts("apply_grid", 2)
        opts("apply_piece_kib", 4)
    if pipeline == "oneshot16":
        opts("apply_grid", 1)
        opts("apply_piece_kib", 16)


@pytest.mark.parametrize("pipeline", ["fused", "unfused", "unfused_fine", "oneshot_loop", "oneshot16"])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("chunk_size", [512, 128 * 1024])
def test_update_batch_vs_replica_oracle(hf, orc, dev, mode, chunk_size, pipeline, opts):
    _set_pipeline(opts, pipeline)
    rng = np.random.default_rng(chunk_size + mode)
    n = 48
    chunks = [bytearray(chunk_size) for _ in range(n)]
    sizes = [0] * n
    cks = [(1, 0)] * n
    dchunks = torch.zeros(n * chunk_size, dtype=torch.uint8, device=dev)
    payload = torch.zeros(n * chunk_size, dtype=torch.uint8, device=dev)
    for rnd in range(12):
        pattern = ["seq", "rand", "mixed"][rnd % 3]
        ios = _random_ios(rng, n, chunk_size, sizes, cks, pattern)
        arr = (hf.UpdateIO * n)()
        host_payload = np.zeros(n * chunk_size, dtype=np.uint8)
        expect = []
        for c, io in enumerate(ios):
            u = arr[c]
            u.chunk = dchunks.data_ptr() + c * chunk_size
            u.chunk_size = sizes[c]
            u.chunk_checksum_type, u.chunk_checksum = cks[c]
            if io[0] == "W":
                _, off, ln = io
                data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
                host_payload[c * chunk_size:c * chunk_size + ln] = np.frombuffer(data, np.uint8)
                wck = orc.create(1, data)
                if rng.random() < 0.05:
                    wck = (1, wck[1] ^ 0x10)  # corrupted client checksum
                u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
                u.payload = payload.data_ptr() + c * chunk_size
                u.write_checksum_type, u.write_checksum = wck
                expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], orc.WRITE, off, ln, data, wck, with_case=True))
            else:
                kind = hf.UPDATE_TRUNCATE if io[0] == "T" else hf.UPDATE_EXTEND
                u.update_type, u.offset, u.length = kind, 0, int(io[1])
                expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], kind, 0, int(io[1]), with_case=True))
        payload.copy_(to_dev(host_payload, dev))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        hf._lib.update_batch(1, d_ios, n, chunk_size, mode=mode, stream=stream())
        torch.cuda.synchronize()
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        hchunks = dchunks.cpu().numpy()
        for c in range(n):
            rc, size, ck, kase = expect[c]
            assert res[c].status == rc, (rnd, c, ios[c])
            assert res[c].checksum_case == kase, (rnd, c, ios[c], mode)  # the reference's counter
            assert res[c].out_size == size, (rnd, c, ios[c])
            assert (res[c].out_checksum_type, res[c].out_checksum) == tuple(ck), (rnd, c, ios[c], mode)
            sizes[c], cks[c] = size, tuple(ck)
            assert bytes(hchunks[c * chunk_size:c * chunk_size + size]) == bytes(chunks[c][:size]), (rnd, c)


@pytest.mark.parametrize("mode", [0, 1])
def test_update_batch_max_chunk_size(hf, orc, dev, mode):
    """Largest chunks the reference has (CHUNK_SIZE_ULTRA = 64 MiB,
    chunk_engine/src/core/constants.rs:6): writes of up to 9 MiB at offsets
    past 32 MiB, appends, gaps past the end and truncates, against
    ChunkReplica::update restated (ChunkReplica.cc:132-394)."""
    rng = np.random.default_rng(640 + mode)
    n, chunk_size = 3, 64 << 20
    chunks = [bytearray(chunk_size) for _ in range(n)]
    sizes, cks = [0] * n, [(1, 0)] * n
    dchunks = torch.zeros(n * chunk_size, dtype=torch.uint8, device=dev)
    payload = torch.zeros(n * (9 << 20), dtype=torch.uint8, device=dev)
    plan = [  # per round: one IO per chunk
        [("W", 0, 9 << 20), ("W", 40 << 20, (3 << 20) + 5), ("W", chunk_size - 7, 7)],
        [("W", 9 << 20, 1 << 20), ("W", 20 << 20, 777), ("T", 33 << 20)],
        [("W", 33 << 20, (5 << 20) + 3), ("E", 50 << 20), ("W", (63 << 20) + 1, (1 << 20) - 1)],
        [("W", 1, (8 << 20) + 11), ("W", 45 << 20, 19 << 20 // 4), ("T", 0)],
    ]
    for rnd, ios in enumerate(plan):
        arr = (hf.UpdateIO * n)()
        host_payload = np.zeros(n * (9 << 20), dtype=np.uint8)
        expect = []
        for c, io in enumerate(ios):
            u = arr[c]
            u.chunk = dchunks.data_ptr() + c * chunk_size
            u.chunk_size = sizes[c]
            u.chunk_checksum_type, u.chunk_checksum = cks[c]
            if io[0] == "W":
                _, off, ln = io
                data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
                host_payload[c * (9 << 20):c * (9 << 20) + ln] = np.frombuffer(data, np.uint8)
                wck = orc.create(1, data)
                u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
                u.payload = payload.data_ptr() + c * (9 << 20)
                u.write_checksum_type, u.write_checksum = wck
                expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], orc.WRITE, off, ln, data, wck, with_case=True))
            else:
                kind = hf.UPDATE_TRUNCATE if io[0] == "T" else hf.UPDATE_EXTEND
                u.update_type, u.offset, u.length = kind, 0, int(io[1])
                expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], kind, 0, int(io[1]), with_case=True))
        payload.copy_(to_dev(host_payload, dev))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        hf._lib.update_batch(1, d_ios, n, chunk_size, mode=mode, stream=stream())
        torch.cuda.synchronize()
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        for c in range(n):
            rc, size, ck, kase = expect[c]
            assert res[c].status == rc, (rnd, c, ios[c])
            assert res[c].checksum_case == kase, (rnd, c, ios[c], mode)  # the reference's counter
            assert res[c].out_size == size, (rnd, c, ios[c])
            assert (res[c].out_checksum_type, res[c].out_checksum) == tuple(ck), (rnd, c, ios[c], mode)
            sizes[c], cks[c] = size, tuple(ck)
            got = dchunks[c * chunk_size:c * chunk_size + size].cpu().numpy().tobytes()
            assert got == bytes(chunks[c][:size]), (rnd, c)
        assert all(r == 0 for r, _, _, _ in expect)


def _run_update_plan(hf, orc, dev, mode, chunk_size, plan, payload_cap, seed):
    """One IO per chunk per round (("W", off, len[, corrupt]), ("T", len), ("E", len)),
    every status / size / checksum / chunk byte against replica_apply."""
    rng = np.random.default_rng(seed)
    n = len(plan[0])
    chunks = [bytearray(chunk_size) for _ in range(n)]
    sizes, cks = [0] * n, [(1, 0)] * n
    dchunks = torch.zeros(n * chunk_size, dtype=torch.uint8, device=dev)
    payload = torch.zeros(n * payload_cap, dtype=torch.uint8, device=dev)
    for rnd, ios in enumerate(plan):
        arr = (hf.UpdateIO * n)()
        host_payload = np.zeros(n * payload_cap, dtype=np.uint8)
        expect = []
        for c, io in enumerate(ios):
            u = arr[c]
            u.chunk = dchunks.data_ptr() + c * chunk_size
            u.chunk_size = sizes[c]
            u.chunk_checksum_type, u.chunk_checksum = cks[c]
            if io[0] == "W":
                off, ln = io[1], io[2]
                data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
                host_payload[c * payload_cap + 3:c * payload_cap + 3 + ln] = np.frombuffer(data, np.uint8)
                wck = orc.create(1, data)
                if len(io) > 3:
                    wck = (1, wck[1] ^ 0x4000)  # corrupted client checksum: chunk untouched
                u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
                u.payload = payload.data_ptr() + c * payload_cap + 3  # misaligned source
                u.write_checksum_type, u.write_checksum = wck
                expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], orc.WRITE, off, ln, data, wck, with_case=True))
            else:
                kind = hf.UPDATE_TRUNCATE if io[0] == "T" else hf.UPDATE_EXTEND
                u.update_type, u.offset, u.length = kind, 0, int(io[1])
                expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], kind, 0, int(io[1]), with_case=True))
        payload.copy_(to_dev(host_payload, dev))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        hf._lib.update_batch(1, d_ios, n, chunk_size, mode=mode, stream=stream())
        torch.cuda.synchronize()
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        for c in range(n):
            rc, size, ck, kase = expect[c]
            assert res[c].status == rc, (rnd, c, ios[c])
            assert res[c].checksum_case == kase, (rnd, c, ios[c], mode)  # the reference's counter
            assert res[c].out_size == size, (rnd, c, ios[c])
            assert (res[c].out_checksum_type, res[c].out_checksum) == tuple(ck), (rnd, c, ios[c], mode)
            sizes[c], cks[c] = size, tuple(ck)
            got = dchunks[c * chunk_size:c * chunk_size + size].cpu().numpy().tobytes()
            assert got == bytes(chunks[c][:size]), (rnd, c)


@pytest.mark.parametrize("pipeline", ["fused", "unfused"])
def test_update_delta_8MiB_chunks(hf, orc, dev, pipeline, opts):
    """DELTA on 8 MiB chunks (up to 130 apply pieces of 64 KiB per IO): whole-chunk
    writes, multi-MiB writes at odd
    offsets, appends, gaps past the end, truncates and extends, corrupted client
    checksums (chunk untouched), misaligned payloads, vs ChunkReplica::update
    restated (ChunkReplica.cc:132-394)."""
    _set_pipeline(opts, pipeline)
    M = 1 << 20
    cs = 8 * M
    plan = [
        [("W", 0, cs), ("W", 5, 3 * M + 7), ("W", 0, 65536), ("W", 123, 1), ("W", 0, 4 * M, 1), ("E", 70000)],
        [("W", 1, cs - 1), ("W", 3 * M + 12, M), ("W", 65536 + 5000, 2 * M), ("W", 124, 65535), ("W", 0, 4 * M),
         ("W", 70000, 131072)],
        [("T", 3 * M + 1), ("W", 7 * M, M - 3), ("W", 2 * M + 65536 + 5000, 65535, 1), ("E", cs),
         ("W", M + 17, 3 * M), ("W", 201000 + 4093, 17)],
        [("W", 3 * M + 1, 4 * M + 2), ("T", 0), ("W", 65535, 2), ("W", cs - 16, 16), ("T", 4 * M - 1),
         ("W", 201000 + 4110, 7 * M)],
    ]
    _run_update_plan(hf, orc, dev, 1, cs, plan, cs + 64, 808)


def _update_round(hf, orc, rng, ios, arr, dchunks, chunks, sizes, cks, cs, payload_base, host_payload):
    """Fill arr / host_payload for one round of _random_ios; returns the replica_apply expectations."""
    expect = []
    for c, io in enumerate(ios):
        u = arr[c]
        u.chunk = dchunks.data_ptr() + c * cs
        u.chunk_size = sizes[c]
        u.chunk_checksum_type, u.chunk_checksum = cks[c]
        if io[0] == "W":
            _, off, ln = io
            data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            host_payload[c * cs:c * cs + ln] = np.frombuffer(data, np.uint8)
            wck = orc.create(1, data)
            if rng.random() < 0.05:
                wck = (1, wck[1] ^ 0x800)  # corrupted client checksum: a real mismatch, the audit keeps 4080
            u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
            u.payload = payload_base + c * cs
            u.write_checksum_type, u.write_checksum = wck
            expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], orc.WRITE, off, ln, data, wck, with_case=True))
        else:
            kind = hf.UPDATE_TRUNCATE if io[0] == "T" else hf.UPDATE_EXTEND
            u.update_type, u.offset, u.length = kind, 0, int(io[1])
            expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], kind, 0, int(io[1]), with_case=True))
    return expect


POISON = [0xFFFFFFFF, 0x80000000, 0x00000001, 0x5A5A5A5A, 0xDEADBEEF, 0x0000FFFF]


@pytest.mark.parametrize("captured", [False, True], ids=["pair_buffer", "captured"])
@pytest.mark.parametrize("pipeline", ["fused", "unfused"])
@pytest.mark.parametrize("mode", [0, 1])
def test_update_batch_poisoned_scratch(hf, orc, dev, mode, pipeline, captured, opts):
    """Incident guard: every library scratch word an update batch gets is first
    set to junk (option poison: a fill kernel on the call's stream right before the pipeline,
    inside the graph when captured), a different pattern every batch.  Outside a capture the
    words are the (stream, thread) pair's own buffer; under capture (torch.cuda.graph, no
    warm-up call) the captured call's own buffer, poisoned at every replay.  Every status,
    case, size, checksum and chunk byte must match ChunkReplica::update restated, and the
    self-check must find nothing: no word of the call is read before the call writes it."""
    _set_pipeline(opts, pipeline)
    L = hf._lib
    L.anomalies(0, reset=True)
    st = torch.cuda.Stream(dev)
    rng = np.random.default_rng(4080 + 2 * mode + captured)
    n, cs = 64, 128 * 1024
    chunks = [bytearray(cs) for _ in range(n)]
    sizes, cks = [0] * n, [(1, 0)] * n
    dchunks = torch.zeros(n * cs, dtype=torch.uint8, device=dev)
    payload = torch.zeros(n * cs, dtype=torch.uint8, device=dev)
    d_ios = torch.zeros(n * ctypes.sizeof(hf.UpdateIO), dtype=torch.uint8, device=dev)
    for rnd in range(6):
        opts("poison", POISON[rnd])
        ios = _random_ios(rng, n, cs, sizes, cks, ["seq", "rand", "mixed"][rnd % 3])
        arr = (hf.UpdateIO * n)()
        host_payload = np.zeros(n * cs, dtype=np.uint8)
        expect = _update_round(hf, orc, rng, ios, arr, dchunks, chunks, sizes, cks, cs, payload.data_ptr(),
                               host_payload)
        payload.copy_(to_dev(host_payload, dev))
        d_ios.copy_(torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev))
        torch.cuda.synchronize()
        if captured:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                L.update_batch(1, d_ios, n, cs, mode=mode, stream=torch.cuda.current_stream())
            g.replay()
            torch.cuda.synchronize()
            del g
        else:
            L.update_batch(1, d_ios, n, cs, mode=mode, stream=st)
            st.synchronize()
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        h = dchunks.cpu().numpy()
        for c in range(n):
            rc, size, ck, kase = expect[c]
            assert res[c].status == rc, (rnd, c, ios[c])
            assert res[c].checksum_case == kase, (rnd, c, ios[c])
            assert res[c].out_size == size, (rnd, c, ios[c])
            assert (res[c].out_checksum_type, res[c].out_checksum) == tuple(ck), (rnd, c, ios[c], mode)
            sizes[c], cks[c] = size, tuple(ck)
            assert bytes(h[c * cs:c * cs + size]) == bytes(chunks[c][:size]), (rnd, c)
    assert L.anomalies(0)["count"] == 0
    if captured:
        L.release_graph_scratch()


@pytest.mark.parametrize("rep", ["1", "3"], ids=["one_run", "prehash_rep3"])
def test_update_one_shot_hint_across_release_stream(hf, orc, dev, rep, opts):
    """The one-shot apply's grid comes from the (stream, thread) pair's previous call (a pinned
    hint word); the pair's first call takes the ticketed apply.  A fresh stream: batches of
    varying size (the grid scaled from the previous call's pieces per IO, short or long of the
    count), release_stream in between (the pair's hint word cleared and recycled: the next call
    is a first call again), every result vs ChunkReplica::update restated; also with the pre
    hash in three byte runs per wave (option prehash_rep)."""
    _set_pipeline(opts, "unfused")
    opts("prehash_rep", rep)
    L = hf._lib
    L.anomalies(0, reset=True)
    st = torch.cuda.Stream(dev)
    rng = np.random.default_rng(4090)
    nmax, cs = 200, 128 * 1024
    chunks = [bytearray(cs) for _ in range(nmax)]
    sizes, cks = [0] * nmax, [(1, 0)] * nmax
    dchunks = torch.zeros(nmax * cs, dtype=torch.uint8, device=dev)
    payload = torch.zeros(nmax * cs, dtype=torch.uint8, device=dev)
    for rnd, (n, release) in enumerate([(64, False), (200, False), (9, True), (150, False), (150, True), (40, False)]):
        ios = _random_ios(rng, n, cs, sizes[:n], cks[:n], ["seq", "rand", "mixed"][rnd % 3])
        arr = (hf.UpdateIO * n)()
        host_payload = np.zeros(n * cs, dtype=np.uint8)
        expect = _update_round(hf, orc, rng, ios, arr, dchunks, chunks[:n], sizes[:n], cks[:n], cs,
                               payload.data_ptr(), host_payload)
        payload[:n * cs].copy_(to_dev(host_payload, dev))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        torch.cuda.synchronize()
        L.update_batch(1, d_ios, n, cs, mode=1, stream=st)
        st.synchronize()
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        h = dchunks.cpu().numpy()
        for c in range(n):
            rc, size, ck, kase = expect[c]
            assert res[c].status == rc, (rnd, c, ios[c])
            assert res[c].checksum_case == kase, (rnd, c, ios[c])
            assert res[c].out_size == size, (rnd, c, ios[c])
            assert (res[c].out_checksum_type, res[c].out_checksum) == tuple(ck), (rnd, c, ios[c])
            sizes[c], cks[c] = size, tuple(ck)
            assert bytes(h[c * cs:c * cs + size]) == bytes(chunks[c][:size]), (rnd, c)
        if release:
            L.release_stream(st)
    assert L.anomalies(0)["count"] == 0


@pytest.mark.parametrize("captured", [False, True], ids=["pair_buffer", "captured"])
def test_update_incident_io_poisoned(hf, orc, dev, captured, opts):
    """The incident's exact IO (scripts/probe_first_call.cpp, tests/cpp/test_checksuminfo.cpp's first
    DELTA update): 232 bytes written at offset 0 of an empty 512-byte chunk with their correct
    checksum, n = 1 -- the pre hash's byte runs then give 232 one-byte parts to 4096 waves.  Both
    modes, both pipelines, every poison pattern, on the null stream; each must verify and set the
    chunk checksum to the payload's."""
    L = hf._lib
    L.anomalies(0, reset=True)
    data = np.random.default_rng(513).integers(0, 256, 232, dtype=np.uint8)
    want = orc.crc32c_raw(data.tobytes())
    dchunk = torch.zeros(512, dtype=torch.uint8, device=dev)
    dpay = to_dev(data, dev)
    d_io = torch.zeros(ctypes.sizeof(hf.UpdateIO), dtype=torch.uint8, device=dev)
    io = hf.UpdateIO()
    io.chunk, io.payload, io.offset, io.length = dchunk.data_ptr(), dpay.data_ptr(), 0, 232
    io.update_type, io.write_checksum_type, io.write_checksum = hf.UPDATE_WRITE, 1, want
    rec = torch.from_numpy(np.frombuffer(bytes(io), dtype=np.uint8).copy()).to(dev)
    st = torch.cuda.Stream(dev)
    for pipeline in ("unfused", "fused"):
        opts("update_pipeline", pipeline)
        for mode in (1, 0):
            for pat in POISON:
                opts("poison", pat)
                dchunk.zero_()
                d_io.copy_(rec)
                torch.cuda.synchronize()
                if captured:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        L.update_batch(1, d_io, 1, 512, mode=mode, stream=torch.cuda.current_stream())
                    g.replay()
                    torch.cuda.synchronize()
                    del g
                else:
                    L.update_batch(1, d_io, 1, 512, mode=mode, stream=None)
                    torch.cuda.synchronize()
                r = hf.UpdateIO.from_buffer_copy(d_io.cpu().numpy().tobytes())
                assert (r.status, r.out_size, r.out_checksum, r.checksum_case) == (0, 232, want, 2), (pipeline, mode,
                                                                                                      hex(pat))
                assert bytes(dchunk[:232].cpu().numpy()) == data.tobytes()
    assert L.anomalies(0)["count"] == 0
    if captured:
        L.release_graph_scratch()


@pytest.mark.parametrize("ctype", [1, 2], ids=["crc32c", "crc32"])
@pytest.mark.parametrize("pipeline", ["fused", "unfused"])
def test_update_audit_contradicts_wrong_verdict(hf, orc, dev, pipeline, ctype, opts):
    """The self-check end to end: option fault_io makes IO 2's pipeline hash start
    from ~0 ^ 1, so its verify fails although the client checksum is right.  The audit re-hashes
    the payload independently, finds the client checksum, and reports the IO as
    HF3FS_CRC_DEVICE_ERROR (chunk untouched) with a PAYLOAD_HASH anomaly naming the IO and both
    values; IO 5's corrupted client checksum stays a real 4080 and every other IO applies.  With
    the audit off the same fault is an (unexplained) 4080.  Both checksum types: the audit's
    CRC32 re-hash uses the CRC32 tables (DeviceTables sh[1])."""
    _set_pipeline(opts, pipeline)
    L = hf._lib
    n, cs = 8, 64 * 1024
    rng = np.random.default_rng(9001)
    for audit in (1, 0):
        opts("audit", audit)
        opts("fault_io", 3)
        L.anomalies(0, reset=True)
        dchunks = torch.zeros(n * cs, dtype=torch.uint8, device=dev)
        payload = torch.zeros(n * cs, dtype=torch.uint8, device=dev)
        arr = (hf.UpdateIO * n)()
        host = np.zeros(n * cs, dtype=np.uint8)
        wcks = []
        for c in range(n):
            ln = int(rng.integers(1000, cs))
            data = rng.integers(0, 256, ln, dtype=np.uint8)
            host[c * cs:c * cs + ln] = data
            wck = (orc.crc32c_raw if ctype == 1 else orc.crc32_raw)(data.tobytes())
            wcks.append(wck)
            u = arr[c]
            u.chunk, u.payload, u.offset, u.length = dchunks.data_ptr() + c * cs, payload.data_ptr() + c * cs, 0, ln
            u.update_type, u.write_checksum_type = hf.UPDATE_WRITE, ctype
            u.write_checksum = wck ^ (0x40 if c == 5 else 0)
        payload.copy_(to_dev(host, dev))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        L.update_batch(ctype, d_ios, n, cs, mode=1, stream=stream())
        torch.cuda.synchronize()
        opts("fault_io", 0)
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        h = dchunks.cpu().numpy()
        for c in range(n):
            if c == 2:
                assert res[c].status == (hf.DEVICE_ERROR if audit else hf.CHECKSUM_MISMATCH)
                assert res[c].out_size == 0 and not h[c * cs:(c + 1) * cs].any()  # chunk untouched
            elif c == 5:
                assert res[c].status == hf.CHECKSUM_MISMATCH
            else:
                assert (res[c].status, res[c].out_checksum) == (0, wcks[c])
        a = L.anomalies(0, reset=True)
        if audit:
            assert a["count"] == 1 and a["kinds"] == a["kind"] == hf._lib.ANOMALY_PAYLOAD_HASH, a
            assert (a["io"], a["rehash"], a["client_checksum"]) == (2, wcks[2], wcks[2]), a
            raw = orc.crc32c_raw if ctype == 1 else orc.crc32_raw
            assert a["pipeline_hash"] == raw(host[2 * cs:2 * cs + arr[2].length].tobytes(), 0xFFFFFFFE)
            assert (a["payload"], a["length"], a["pre_len"]) == (arr[2].payload, arr[2].length, arr[2].length)
            assert a["pipeline"] == (0 if pipeline == "unfused" else 1) | (1 << 8)
        else:
            assert a["count"] == 0


@pytest.mark.parametrize("mode", [0, 1])
def test_update_d3_shape(hf, orc, dev, mode):
    """BASELINE configs[2] at its shape: 1024 resident 4 MiB chunks, one write per
    chunk per batch of U[64 KiB, 1 MiB] at byte offsets, 10 % appends, 5 % writes
    past the end with a zero-filled gap, 1 % corrupted client checksums, on the
    library's default pipeline for the mode (REFERENCE: fused; DELTA: three-pass).
    After every batch EVERY chunk's status, size, checksum (== CRC32C of its bytes,
    the invariant TestStorageClientInterface.cc:433-435 asserts) and bytes are
    checked against a host model."""
    n, cs, M = 1024, 4 << 20, 1 << 20
    rng = np.random.default_rng(31 + mode)
    model = np.zeros((n, cs), dtype=np.uint8)
    sizes = rng.integers(2 * M, cs + 1, n)
    dchunks = torch.empty(n * cs, dtype=torch.uint8, device=dev)
    hf._lib.fill_synth(dchunks, cs, cs, n, SEED, 0, stream=stream())
    torch.cuda.synchronize()
    model[:] = dchunks.view(n, cs).cpu().numpy()
    cks = np.array([orc.crc32c_raw(model[c, :sizes[c]]) for c in range(n)], dtype=np.uint64)
    payload = torch.empty(n * M, dtype=torch.uint8, device=dev)
    for batch in range(3):
        lens = rng.integers(64 << 10, M + 1, n)
        offs = np.array([rng.integers(0, cs - ln + 1) for ln in lens])
        r = rng.random(n)
        app = (r < 0.10) & (sizes + lens <= cs)
        offs[app] = sizes[app]
        gap = (r >= 0.10) & (r < 0.15) & (sizes + lens + 4096 <= cs)
        offs[gap] = sizes[gap] + rng.integers(1, 4097, gap.sum())
        bad = rng.random(n) < 0.01
        hf._lib.fill_synth(payload, M, M, n, SEED ^ (0x51 + batch), 7 * batch, stream=stream())
        torch.cuda.synchronize()
        hp = payload.view(n, M).cpu().numpy()
        arr = (hf.UpdateIO * n)()
        for c in range(n):
            u = arr[c]
            u.chunk = dchunks.data_ptr() + c * cs
            u.payload = payload.data_ptr() + c * M
            u.offset, u.length, u.chunk_size = int(offs[c]), int(lens[c]), int(sizes[c])
            u.update_type = hf.UPDATE_WRITE
            u.chunk_checksum_type, u.chunk_checksum = hf.CRC32C, int(cks[c])
            wck = orc.crc32c_raw(hp[c, :lens[c]])
            u.write_checksum_type, u.write_checksum = hf.CRC32C, (wck ^ (0x20 if bad[c] else 0))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        hf._lib.update_batch(1, d_ios, n, cs, mode=mode, stream=stream())
        torch.cuda.synchronize()
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        kase = np.zeros(n, dtype=np.int64)  # ChunkReplica.cc:334-389: reuse / combine (append) / read_chunk
        for c in range(n):  # the host model: gap zero-fill, then the payload (ChunkReplica.cc:281-292)
            if bad[c]:
                continue
            o, ln = int(offs[c]), int(lens[c])
            s1 = max(int(sizes[c]), o + ln)
            kase[c] = 2 if (o == 0 and ln == s1) else 3 if (o == sizes[c] and sizes[c] > 0) else 4
            if o > sizes[c]:
                model[c, sizes[c]:o] = 0
            model[c, o:o + ln] = hp[c, :ln]
            sizes[c] = max(int(sizes[c]), o + ln)
        back = dchunks.view(n, cs).cpu().numpy()
        for c in range(n):
            assert res[c].status == (4080 if bad[c] else 0), (batch, c)
            assert res[c].checksum_case == kase[c], (batch, c)
            assert res[c].out_size == sizes[c], (batch, c)
            want = orc.crc32c_raw(model[c, :sizes[c]])
            assert res[c].out_checksum == want, (batch, c, mode)
            cks[c] = want
            assert np.array_equal(back[c, :sizes[c]], model[c, :sizes[c]]), (batch, c)
    del dchunks, payload
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pipeline", ["fused", "unfused"])
@pytest.mark.parametrize("mode", [0, 1])
def test_update_mixed_chunk_types(hf, orc, dev, mode, pipeline, opts):
    """A write whose checksum type differs from the chunk's (ChunkReplica.cc:340,
    356-392): CRC32 and NONE-typed chunks with data receive CRC32C writes in a
    CRC32C batch -- the prefix and suffix are recomputed in CRC32C and the chunk
    takes the write's type; appends of a different type do not combine; a
    NONE-typed write resets the chunk to {NONE, 0}.  A truncate / extend hashes
    in the chunk's type: a CRC32 chunk's truncate runs in a CRC32 batch (in a
    CRC32C batch it is kInvalidArg, include/hf3fs_crc.h)."""
    _set_pipeline(opts, pipeline)
    rng = np.random.default_rng(55 + mode)
    n, cs = 24, 64 * 1024
    chunks = [bytearray(rng.integers(0, 256, cs, dtype=np.uint8).tobytes()) for _ in range(n)]
    sizes = [int(rng.integers(1, cs)) for _ in range(n)]
    cks = []
    for c in range(n):
        t = [2, 2, 0, 1][c % 4]
        cks.append(orc.create(t, bytes(chunks[c][:sizes[c]])) if t else (0, 0))
    dchunks = to_dev(np.frombuffer(b"".join(bytes(x) for x in chunks), np.uint8).copy(), dev)
    payload = torch.zeros(n * cs, dtype=torch.uint8, device=dev)

    def run(batch_type, plan):
        arr = (hf.UpdateIO * n)()
        host_payload = np.zeros(n * cs, dtype=np.uint8)
        expect = []
        for c, io in enumerate(plan):
            u = arr[c]
            u.chunk = dchunks.data_ptr() + c * cs
            u.chunk_size = sizes[c]
            u.chunk_checksum_type, u.chunk_checksum = cks[c]
            if io[0] == "W":
                _, off, ln, wt = io
                data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
                host_payload[c * cs:c * cs + ln] = np.frombuffer(data, np.uint8)
                wck = orc.create(wt, data) if wt else (0, 0)
                u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
                u.payload = payload.data_ptr() + c * cs
                u.write_checksum_type, u.write_checksum = wck
                expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], orc.WRITE, off, ln, data, wck, with_case=True))
            elif io[0] == "X":  # not part of this batch: an extend to the current size is a no-op
                u.update_type, u.offset, u.length = hf.UPDATE_EXTEND, 0, sizes[c]
                expect.append(None)
            else:
                kind = hf.UPDATE_TRUNCATE if io[0] == "T" else hf.UPDATE_EXTEND
                u.update_type, u.offset, u.length = kind, 0, int(io[1])
                if cks[c][0] not in (0, batch_type):
                    expect.append((3, sizes[c], cks[c], 0))  # hashes in the chunk's type: other batch
                else:
                    expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], kind, 0, int(io[1]), with_case=True))
        payload.copy_(to_dev(host_payload, dev))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        hf._lib.update_batch(batch_type, d_ios, n, cs, mode=mode, stream=stream())
        torch.cuda.synchronize()
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        for c in range(n):
            if expect[c] is None:
                continue
            rc, size, ck, kase = expect[c]
            assert res[c].status == rc, (c, plan[c], cks[c])
            assert res[c].checksum_case == kase, (c, plan[c], cks[c], mode)
            if rc:
                continue
            assert res[c].out_size == size, (c, plan[c])
            assert (res[c].out_checksum_type, res[c].out_checksum) == tuple(ck), (c, plan[c], cks[c], mode)
            sizes[c], cks[c] = size, tuple(ck)
            got = dchunks[c * cs:c * cs + size].cpu().numpy().tobytes()
            assert got == bytes(chunks[c][:size]), c

    # round 1, CRC32C batch: writes of every kind into chunks of every type
    plan = []
    for c in range(n):
        k = c % 6
        if k == 0:
            plan.append(("W", int(rng.integers(0, sizes[c])), int(rng.integers(1, 9000)), 1))  # overwrite inside
        elif k == 1:
            plan.append(("W", sizes[c], int(rng.integers(1, cs - sizes[c] + 1)), 1))  # append, other type
        elif k == 2:
            plan.append(("W", 0, cs, 1))  # full overwrite: reuse
        elif k == 3:
            plan.append(("W", int(rng.integers(0, sizes[c])), 100, 0))  # NONE-typed write
        elif k == 4:
            plan.append(("T", int(rng.integers(0, sizes[c] + 1))))  # truncate: chunk type vs batch type
        else:
            plan.append(("W", sizes[c] + 77, 500, 1))  # gap write
    plan = [p if (p[0] != "W" or p[1] + p[2] <= cs) else ("W", p[1], cs - p[1], p[3]) for p in plan]
    run(1, plan)
    # round 2, CRC32 batch: the truncates / extends of chunks still typed CRC32 (or NONE)
    plan2 = [("T", max(0, sizes[c] - 1000)) if cks[c][0] in (0, 2) else ("X",) for c in range(n)]
    run(2, plan2)


# ---- chunk-engine semantics (HF3FS_UPDATE_FLAG_ENGINE) vs the Rust-engine restatement ---------
@pytest.mark.parametrize("pipeline", ["fused", "unfused", "unfused_fine", "oneshot_loop"])
@pytest.mark.parametrize("mode", [0, 1])
def test_update_engine_flag_vs_engine_oracle(hf, orc, dev, mode, pipeline, opts):
    _set_pipeline(opts, pipeline)
    rng = np.random.default_rng(77 + mode)
    n, cap = 32, 64 * 1024
    bufs = [bytearray(cap) for _ in range(n)]
    lens, fins, exists = [0] * n, [0] * n, [False] * n
    dchunks = torch.zeros(n * cap, dtype=torch.uint8, device=dev)
    payload = torch.zeros(n * cap, dtype=torch.uint8, device=dev)
    for rnd in range(14):
        arr = (hf.UpdateIO * n)()
        host_payload = np.zeros(n * cap, dtype=np.uint8)
        expect = []
        for c in range(n):
            u = arr[c]
            u.chunk = dchunks.data_ptr() + c * cap
            u.chunk_size = lens[c]
            u.chunk_checksum_type, u.chunk_checksum = hf.CRC32C, (~fins[c]) & M32
            u.flags = hf._lib.UPDATE_FLAG_ENGINE
            r = rng.random()
            if exists[c] and r < 0.15:  # truncate / extend to a target length (bridge: req.offset = length)
                target = int(rng.integers(0, cap + 1))
                trunc = r < 0.10
                u.update_type = hf.UPDATE_TRUNCATE if trunc else hf.UPDATE_EXTEND
                u.length = target
                expect.append(orc.engine_apply(bufs[c], lens[c], fins[c], b"", target, cap, truncate=trunc,
                                               with_case=True))
                continue
            off = lens[c] if r < 0.45 else int(rng.integers(0, min(cap - 1, lens[c] + 5000) + 1))
            ln = int(rng.choice([rng.integers(1, 3000), 4096, 8192]))
            ln = min(ln, cap - off)
            if ln <= 0:
                off, ln = 0, 1
            data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            host_payload[c * cap:c * cap + ln] = np.frombuffer(data, np.uint8)
            fin = orc.rs_crc32c(data)
            without = rng.random() < 0.3
            bad = (not without) and rng.random() < 0.05
            u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
            u.payload = payload.data_ptr() + c * cap
            if without:
                u.write_checksum_type, u.write_checksum = hf.NONE, 0
            else:
                u.write_checksum_type, u.write_checksum = hf.CRC32C, (~fin ^ (0x100 if bad else 0)) & M32
            expect.append(orc.engine_apply(bufs[c], lens[c], fins[c], data, off, cap, exists=exists[c],
                                           data_ck=fin ^ (0x100 if bad else 0), with_case=True))
        payload.copy_(to_dev(host_payload, dev))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        hf._lib.update_batch(1, d_ios, n, cap, mode=mode, stream=stream())
        torch.cuda.synchronize()
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        h = dchunks.cpu().numpy()
        for c in range(n):
            rc, nl, nf, kase = expect[c]
            assert res[c].status == rc, (rnd, c)
            assert res[c].checksum_case == kase, (rnd, c, mode, res[c].update_type, res[c].offset, res[c].length,
                                                  res[c].chunk_size)  # chunk.rs metrics counter
            if rc == 0:
                assert res[c].out_size == nl, (rnd, c)
                assert res[c].out_checksum_type == hf.CRC32C
                r_ = res[c]
                assert (~r_.out_checksum) & M32 == nf, (rnd, c, mode, r_.update_type, r_.offset, r_.length,
                                                        r_.chunk_size, r_.write_checksum_type, r_.out_size)
                assert nf == orc.rs_crc32c(bytes(bufs[c][:nl]))
                assert bytes(h[c * cap:c * cap + nl]) == bytes(bufs[c][:nl]), (rnd, c)
                lens[c], fins[c], exists[c] = nl, nf, True


# ---- AioReadJob::setResult batch ----------------------------------------------------------------
@pytest.mark.parametrize("bound", [128 * 1024, 16 << 20])
def test_read_result_batch_vs_oracle(hf, orc, dev, bound):
    """bound = the call's max_len (a loose bound must not change any result)."""
    rng = np.random.default_rng(12)
    n, cl = 200, 128 * 1024
    host = rng.integers(0, 256, n * cl, dtype=np.uint8)
    d = to_dev(host, dev)
    arr = (hf._lib.ReadIO * n)()
    expect = []
    for i in range(n):
        chunk = host[i * cl:(i + 1) * cl]
        ck = orc.create(1, chunk)
        stale = rng.random() < 0.1
        stored = (1, ck[1] ^ 0x80) if stale else ck
        full = rng.random() < 0.4
        off = 0 if full else int(rng.integers(0, cl - 1))
        ln = cl if full else int(rng.integers(0, cl - off + 1))
        btype = int(rng.choice([0, 1, 1, 1]))
        recalc = rng.random() < 0.5
        u = arr[i]
        u.data = d.data_ptr() + i * cl + off
        u.offset, u.length, u.chunk_len = off, ln, cl
        u.batch_checksum_type, u.chunk_checksum_type, u.chunk_checksum = btype, stored[0], stored[1]
        u.recalculate = int(recalc)
        expect.append(orc.read_result(btype, stored, off, chunk[off:off + ln], cl, full_chunk=chunk,
                                      recalculate=recalc))
    d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
    hf._lib.read_result_batch(1, d_ios, n, bound, stream=stream())
    torch.cuda.synchronize()
    res = (hf._lib.ReadIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
    for i in range(n):
        rc, (t, v) = expect[i]
        assert res[i].status == rc, i
        assert (res[i].out_checksum_type, res[i].out_checksum) == (t, v), i


@pytest.mark.parametrize("batch", [32, 256, 1024])
def test_read_result_batch_registered_host(hf, orc, dev, batch):
    """The read path INTEGRATION.md 2.1 recommends: each worker thread
    reaps a batch of completed reads (AioReadWorker.cc:60-94; batches of up to 1024,
    StorageOperator.cc:163-167) whose bytes AND IO records sit in hf3fs_crc_host_register'ed
    host memory, and runs setResult's checksum part for the batch in one call on its own
    stream.  4 threads x 3 batches of {4..64} KiB reads (partial reads hashed, full-chunk
    reads reused or re-hashed with recalculate against stale stored checksums, NONE
    batches); every record vs orc_read_result_checksum (BatchReadJob.cc:24-63)."""
    import threading
    L = hf._lib
    rng0 = np.random.default_rng(2400 + batch)
    arena = rng0.integers(0, 256, 64 << 20, dtype=np.uint8)
    d_arena = L.host_register(arena.ctypes.data, arena.size)
    threads, rounds = 4, 3
    def page_aligned(nbytes):  # registrations must not share a page
        size = (nbytes + 4095) // 4096 * 4096
        raw = np.zeros(size + 4096, dtype=np.uint8)
        k = (-raw.ctypes.data) % 4096
        return raw[k:k + size]

    recs = [page_aligned(batch * ctypes.sizeof(L.ReadIO)) for _ in range(threads)]
    d_recs = [L.host_register(r.ctypes.data, r.size) for r in recs]
    errors = []

    def work(t):
        try:
            rng = np.random.default_rng(100 * batch + t)
            st = torch.cuda.Stream(dev)
            for rnd in range(rounds):
                arr = (L.ReadIO * batch).from_buffer(recs[t][:batch * ctypes.sizeof(L.ReadIO)])
                expect = []
                for i in range(batch):
                    ln = 4096 << int(rng.integers(0, 5))
                    off = int(rng.integers(0, (arena.size - ln) // 4096)) * 4096
                    data = arena[off:off + ln]
                    full = rng.random() < 0.25
                    cl = ln if full else 4 << 20
                    roff = 0 if full else 4096 * int(rng.integers(1, 512))
                    ck = orc.create(1, data.tobytes()) if full else (1, int(rng.integers(0, 1 << 32)))
                    if full and rng.random() < 0.3:
                        ck = (1, ck[1] ^ 0x1000)  # stale stored checksum: recalculate reports 4080
                    btype = int(rng.choice([0, 1, 1, 1]))
                    recalc = full and rng.random() < 0.5
                    u = arr[i]
                    u.data, u.offset, u.length, u.chunk_len = d_arena + off, roff, ln, cl
                    u.batch_checksum_type, u.chunk_checksum_type, u.chunk_checksum = btype, ck[0], ck[1]
                    u.recalculate, u.status, u.out_checksum, u.out_checksum_type = int(recalc), -1, 0, 0
                    expect.append(orc.read_result(btype, ck, roff, data.tobytes(), cl, full_chunk=data.tobytes(),
                                                  recalculate=recalc))
                del arr
                L.read_result_batch(1, d_recs[t], batch, 64 << 10, stream=st)
                st.synchronize()
                res = (L.ReadIO * batch).from_buffer_copy(recs[t][:batch * ctypes.sizeof(L.ReadIO)].tobytes())
                for i in range(batch):
                    rc, (ty, v) = expect[i]
                    if (res[i].status, res[i].out_checksum_type, res[i].out_checksum) != (rc, ty, v):
                        errors.append((t, rnd, i, res[i].status, rc, res[i].out_checksum, v))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    torch.cuda.synchronize()
    for r in recs:
        L.host_unregister(r.ctypes.data)
    L.host_unregister(arena.ctypes.data)
    assert not errors, errors[:5]


@pytest.mark.parametrize("where", ["own_streams", "null_stream"])
def test_update_concurrent_threads_call_scratch(hf, orc, dev, where):
    """Batch calls run on the calling (stream, thread)'s persistent scratch:
    worker threads updating their own chunks concurrently -- each on its own stream, or all
    on the null stream where their launches interleave -- with batch sizes that grow and
    shrink (the scratch is regrown with a stream synchronize between calls) never see each
    other's control words or hash outputs: every status, case, size, checksum and chunk byte
    of every thread matches ChunkReplica::update restated, in both modes."""
    import threading
    threads, rounds, cs = 4, 6, 16 * 1024
    sizes_n = [8, 64, 16, 128, 4, 96]  # IOs per batch, per round (grows and shrinks)
    nmax = max(sizes_n)
    errors = []
    dchunks = [torch.zeros(nmax * cs, dtype=torch.uint8, device=dev) for _ in range(threads)]
    payloads = [torch.zeros(nmax * cs, dtype=torch.uint8, device=dev) for _ in range(threads)]
    torch.cuda.synchronize()

    def worker(k):
        try:
            rng = np.random.default_rng(700 + k)
            mode = k % 2
            s = torch.cuda.Stream(dev) if where == "own_streams" else None
            chunks = [bytearray(cs) for _ in range(nmax)]
            sizes, cks = [0] * nmax, [(1, 0)] * nmax
            for rnd in range(rounds):
                n = sizes_n[(rnd + k) % len(sizes_n)]
                ios = _random_ios(rng, n, cs, sizes, cks, ["seq", "rand", "mixed"][rnd % 3])
                arr = (hf.UpdateIO * n)()
                host_payload = np.zeros(n * cs, dtype=np.uint8)
                expect = []
                for c, io in enumerate(ios):
                    u = arr[c]
                    u.chunk = dchunks[k].data_ptr() + c * cs
                    u.chunk_size = sizes[c]
                    u.chunk_checksum_type, u.chunk_checksum = cks[c]
                    if io[0] == "W":
                        _, off, ln = io
                        data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
                        host_payload[c * cs:c * cs + ln] = np.frombuffer(data, np.uint8)
                        wck = orc.create(1, data)
                        u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
                        u.payload = payloads[k].data_ptr() + c * cs
                        u.write_checksum_type, u.write_checksum = wck
                        expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], orc.WRITE, off, ln, data, wck,
                                                        with_case=True))
                    else:
                        kind = hf.UPDATE_TRUNCATE if io[0] == "T" else hf.UPDATE_EXTEND
                        u.update_type, u.offset, u.length = kind, 0, int(io[1])
                        expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], kind, 0, int(io[1]),
                                                        with_case=True))
                hp = torch.from_numpy(host_payload)
                d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy())
                if s is None:
                    payloads[k][:n * cs].copy_(hp)
                    d_dev = d_ios.to(dev)
                    torch.cuda.synchronize()
                    hf._lib.update_batch(1, d_dev, n, cs, mode=mode, stream=None)
                    torch.cuda.synchronize()
                else:
                    with torch.cuda.stream(s):
                        payloads[k][:n * cs].copy_(hp)
                        d_dev = d_ios.to(dev)
                    hf._lib.update_batch(1, d_dev, n, cs, mode=mode, stream=s)
                    s.synchronize()
                res = (hf.UpdateIO * n).from_buffer_copy(d_dev.cpu().numpy().tobytes())
                hchunks = dchunks[k].cpu().numpy()
                for c in range(n):
                    rc, size, ck, kase = expect[c]
                    got = (res[c].status, res[c].checksum_case, res[c].out_size,
                           (res[c].out_checksum_type, res[c].out_checksum))
                    if got != (rc, kase, size, tuple(ck)) or \
                            bytes(hchunks[c * cs:c * cs + size]) != bytes(chunks[c][:size]):
                        errors.append((k, rnd, c, ios[c], got, (rc, kase, size, tuple(ck))))
                        return
                    sizes[c], cks[c] = size, tuple(ck)
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:3]


@pytest.mark.parametrize("apply", ["default", "oneshot"])
@pytest.mark.parametrize("mode", [0, 1])
def test_update_batch_graph_captured(hf, orc, dev, mode, apply, opts):
    """An update batch captured into a hipGraph (during a capture the call's
    scratch is a stream-ordered allocation the graph owns) and replayed from restored inputs
    gives the same statuses, cases, sizes, checksums and chunk bytes as ChunkReplica::update
    restated.  (An update is not idempotent -- DELTA reads the old bytes it overwrites -- so
    every replay starts from the saved chunks and IO records.)  "oneshot": the three-pass
    pipeline with the one-shot apply, whose finalize is forked onto the pair's side stream and
    joined back inside the capture."""
    if apply == "oneshot":
        opts("update_pipeline", "unfused")
        opts("apply_grid", 1)
    rng = np.random.default_rng(90 + mode)
    n, cs = 32, 64 * 1024
    chunks = [bytearray(cs) for _ in range(n)]
    sizes, cks = [0] * n, [(1, 0)] * n
    dchunks = torch.zeros(n * cs, dtype=torch.uint8, device=dev)
    payload = torch.zeros(n * cs, dtype=torch.uint8, device=dev)
    # a first, uncaptured batch gives the chunks content and checksums
    for rnd in range(2):
        ios = _random_ios(rng, n, cs, sizes, cks, ["seq", "rand"][rnd])
        arr = (hf.UpdateIO * n)()
        host_payload = np.zeros(n * cs, dtype=np.uint8)
        expect = []
        for c, io in enumerate(ios):
            u = arr[c]
            u.chunk = dchunks.data_ptr() + c * cs
            u.chunk_size = sizes[c]
            u.chunk_checksum_type, u.chunk_checksum = cks[c]
            _, off, ln = io
            data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            host_payload[c * cs:c * cs + ln] = np.frombuffer(data, np.uint8)
            wck = orc.create(1, data)
            u.update_type, u.offset, u.length = hf.UPDATE_WRITE, off, ln
            u.payload = payload.data_ptr() + c * cs
            u.write_checksum_type, u.write_checksum = wck
            expect.append(orc.replica_apply(chunks[c], sizes[c], cks[c], orc.WRITE, off, ln, data, wck,
                                            with_case=True))
        payload.copy_(to_dev(host_payload, dev))
        d_ios = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        torch.cuda.synchronize()
        if rnd == 0:
            hf._lib.update_batch(1, d_ios, n, cs, mode=mode, stream=stream())
            torch.cuda.synchronize()
        else:
            saved_chunks, saved_ios = dchunks.clone(), d_ios.clone()
            cap = torch.cuda.Stream(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                hf._lib.update_batch(1, d_ios, n, cs, mode=mode, stream=torch.cuda.current_stream())
            for _ in range(3):  # replays from the restored inputs
                dchunks.copy_(saved_chunks)
                d_ios.copy_(saved_ios)
                torch.cuda.synchronize()
                g.replay()
                torch.cuda.synchronize()
                res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
                hchunks = dchunks.cpu().numpy()
                for c in range(n):
                    rc, size, ck, kase = expect[c]
                    assert (res[c].status, res[c].checksum_case, res[c].out_size) == (rc, kase, size), (c, ios[c])
                    assert (res[c].out_checksum_type, res[c].out_checksum) == tuple(ck), (c, ios[c], mode)
                    assert bytes(hchunks[c * cs:c * cs + size]) == bytes(chunks[c][:size]), c
            del g
        res = (hf.UpdateIO * n).from_buffer_copy(d_ios.cpu().numpy().tobytes())
        for c in range(n):
            rc, size, ck, kase = expect[c]
            assert res[c].status == rc, (rnd, c)
            sizes[c], cks[c] = size, tuple(ck)


def test_stream_wait_polled(hf, orc, dev):
    """hf3fs_crc_stream_wait: a polled, non-spinning wait returns only after the stream's
    queued hash (the bytes' digests are there), and poll_us = 0 is hipStreamSynchronize."""
    n, length = 64, 1 << 20
    buf = torch.empty(n * length, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    hf._lib.fill_synth(buf, length, length, n, SEED, 3, stream=st)
    for poll in (20, 0):
        out.zero_()
        st.wait_stream(torch.cuda.current_stream())
        hf._lib.create_strided(1, buf, length, length, n, out, stream=st)
        hf._lib.stream_wait(st, poll)
        h = out.cpu().numpy().astype(np.uint32)  # (the default stream: no sync with st)
        assert all(int(h[i]) == orc.crc32c_raw(orc.fill_synth(length, SEED, 3 + i)) for i in (0, 31, 63)), poll
