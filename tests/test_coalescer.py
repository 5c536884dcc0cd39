"""GPU parity of the per-IO request coalescer.

Many threads submit single ChecksumInfo::create requests, as 3FS's 32
AioReadWorker / UpdateWorker threads do per IO (BatchReadJob.cc:24-35,
ChunkReplica.cc:193-207); every value must equal the oracle's create over the
same bytes, whether the bytes sit in HBM, in registered host memory (zero
copy) or in plain host memory copied into the pinned stage.
"""
import ctypes
import random
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
M32 = 0xFFFFFFFF


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _requests(rng, arena_len, count):
    """(offset, length, start, type) tuples; lengths cover 0, tiny, KV-block and >1 MiB sizes."""
    out = []
    for _ in range(count):
        r = rng.random()
        if r < 0.05:
            ln = 0
        elif r < 0.3:
            ln = rng.randrange(1, 200)
        elif r < 0.95:
            ln = rng.choice([4, 8, 16, 32, 64]) * 1024 + rng.randrange(-3, 4)
        else:
            ln = rng.randrange(1 << 20, 3 << 20)
        off = rng.randrange(0, arena_len - ln)
        start = M32 if rng.random() < 0.7 else rng.getrandbits(32)
        ctype = 2 if rng.random() < 0.15 else 1
        out.append((off, ln, start, ctype))
    return out


def _run_threads(nthreads, fn):
    errs = []

    def wrap(t):
        try:
            fn(t)
        except BaseException as e:  # noqa: BLE001 - surfaced below
            errs.append(e)

    ths = [threading.Thread(target=wrap, args=(t,)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]


@pytest.mark.parametrize("service_wgs", [0, 8])
@pytest.mark.parametrize("where", ["hbm", "host_copy", "registered"])
def test_threads_create_one_vs_oracle(hf, orc, dev, where, service_wgs):
    L = hf._lib
    rng = np.random.default_rng(7)
    arena_len = 8 << 20
    host = rng.integers(0, 256, arena_len, dtype=np.uint8)
    keep = None
    if where == "hbm":
        d = torch.from_numpy(host).to(dev)
        keep = d
        base = d.data_ptr()
        flags = 0
    elif where == "registered":
        base = L.host_register(host.ctypes.data, arena_len)
        flags = 0
    else:
        base = host.ctypes.data
        flags = L.REQ_HOST_COPY
    results = {}
    nthreads, per = 16, 60
    reqs = {t: _requests(random.Random(100 + t), arena_len, per) for t in range(nthreads)}
    # small stage: exercises full-slot sealing; service mode: small ring exercises slot reuse, and
    # requests over service_stage / CRC32 ones take the batch path beside it
    with L.Coalescer(device=0, stage_bytes=4 << 20, service_wgs=service_wgs, service_ring=64,
                     service_stage=32 << 10) as co:

        def worker(t):
            for k, (off, ln, start, ctype) in enumerate(reqs[t]):
                results[(t, k)] = co.create_one(ctype, base + off, ln, start, flags)

        _run_threads(nthreads, worker)
        st = co.stats()
    if where == "registered":
        L.host_unregister(host.ctypes.data)
    del keep
    for t in range(nthreads):
        for k, (off, ln, start, ctype) in enumerate(reqs[t]):
            want = orc.create(ctype, host[off:off + ln], start)[1]
            assert results[(t, k)] == want, (where, t, k, ln, ctype)
    assert st["batches"] >= 1 and st["requests"] <= nthreads * per


def test_async_submit_drains_on_destroy(hf, orc, dev):
    """Callbacks fire once each with the right value; destroy completes what is pending."""
    L = hf._lib
    rng = np.random.default_rng(11)
    n = 3000
    lens = rng.integers(1, 70000, n)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    host = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    got = {}
    lock = threading.Lock()

    @L.DONE_FN
    def cb(arg, status, value):
        with lock:
            got[arg] = (status, value)

    co = L.Coalescer(device=0, max_batch=512)
    for i in range(n):
        rc = L.load().hf3fs_crc_coalescer_submit(co._h, 1, d.data_ptr() + int(offs[i]), int(lens[i]), M32, 0, cb,
                                                  i + 1)
        assert rc == 0
    st = co.stats()
    co.close()
    assert len(got) == n
    assert st["max_batch"] <= 512
    for i in range(0, n, 7):
        o, ln = int(offs[i]), int(lens[i])
        assert got[i + 1] == (0, orc.crc32c_raw(host[o:o + ln])), i


def test_special_cases_and_large_host_copy(hf, orc, dev):
    L = hf._lib
    data = np.random.default_rng(3).integers(0, 256, (3 << 20) + 5, dtype=np.uint8)
    with L.Coalescer(device=0, stage_bytes=1 << 20) as co:
        assert co.create_one(0, data, 100, flags=L.REQ_HOST_COPY) == 0            # NONE -> {NONE, 0}
        assert co.create_one(1, data, 0, start=0x1234, flags=L.REQ_HOST_COPY) == 0x1234  # len 0 -> start
        big = co.create_one(1, data, data.size, flags=L.REQ_HOST_COPY)             # > stage: staged host path
        assert big == orc.crc32c_raw(data)
        assert co.create_one(2, data, 4097, start=7, flags=L.REQ_HOST_COPY) == \
            orc.create(2, data[:4097], 7)[1]
        with pytest.raises(L.Hf3fsCrcError):
            co.create_one(5, data, 10, flags=L.REQ_HOST_COPY)


def test_options_rejected(hf):
    L = hf._lib
    with pytest.raises(L.Hf3fsCrcError):
        L.Coalescer(device=0, slots=1)
    with pytest.raises(L.Hf3fsCrcError):
        L.Coalescer(device=0, inflight=4, slots=4)


def test_service_async_idle_relaunch(hf, orc, dev):
    """Service mode: every async callback fires once with the right value, and
    requests after the kernel's idle exit relaunch it."""
    import time
    L = hf._lib
    rng = np.random.default_rng(12)
    host = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    got = {}
    lock = threading.Lock()

    @L.DONE_FN
    def cb(arg, status, value):
        with lock:
            got[arg] = (status, value)

    with L.Coalescer(device=0, service_wgs=4, service_ring=128, service_idle_us=500) as co:
        reqs = []
        for rnd in range(3):
            for i in range(300):
                off, ln = int(rng.integers(0, 3 << 20)), int(rng.integers(1, 200000))
                key = len(reqs) + 1
                reqs.append((off, ln))
                assert L.load().hf3fs_crc_coalescer_submit(co._h, 1, d.data_ptr() + off, ln, M32, 0, cb, key) == 0
            v = co.create_one(1, d.data_ptr() + 5, 1000)
            assert v == orc.crc32c_raw(host[5:1005])
            time.sleep(0.05)  # > idle timeout: the kernel exits; the next round relaunches it
        st = co.stats()
    assert len(got) == len(reqs)
    for k, (off, ln) in enumerate(reqs):
        assert got[k + 1] == (0, orc.crc32c_raw(host[off:off + ln])), k
    assert st["requests"] >= len(reqs)
