"""File digest: admin `checksum --fill-zero`.

Reference: src/client/cli/admin/FileWrapper.cc:133-160 (per-block zero fill and
ChecksumInfo::combine fold), called per replica by Checksum.cc:43-88.

  - CPU: the oracle's left fold equals create(CRC32C) over the file's bytes with
    holes as zeros (pins the oracle on the create/combine golden vectors);
  - CPU: a Python model of the kernel's associative summary equals the left fold
    on random block sequences at random split points, every type/length corner;
  - GPU: hf3fs_crc_file_digest_batch vs the oracle, bit-exact, status included.
"""
import random

import numpy as np
import pytest

NONE, CRC32C, CRC32 = 0, 1, 2
M32 = 0xFFFFFFFF
BLOCK_DT = np.dtype([("read_len", "<u8"), ("block_len", "<u8"), ("checksum", "<u4"), ("type", "u1"),
                     ("missing", "u1"), ("res", "u1", (2,))])
FILE_DT = np.dtype([("length", "<u8"), ("value", "<u4"), ("type", "u1"), ("res", "u1", (3,)), ("status", "<i4"),
                    ("res2", "<u4")])
assert BLOCK_DT.itemsize == 24 and FILE_DT.itemsize == 24


def make_file(rng, orc, nblocks, max_len=5000, p_hole=0.2, p_missing=0.1):
    """Blocks of real bytes; returns (blocks for the fold, the bytes the digest covers)."""
    blocks, content = [], bytearray()
    for _ in range(nblocks):
        L = rng.randint(1, max_len)
        data = bytes(rng.getrandbits(8) for _ in range(L))
        u = rng.random()
        if u < p_missing:
            blocks.append((0, L, (NONE, 0)))
            content += bytes(L)
        elif u < p_missing + p_hole:
            r = rng.randint(0, L - 1)
            blocks.append((r, L, orc.create(CRC32C, data[:r])))
            content += data[:r] + bytes(L - r)
        else:
            blocks.append((L, L, orc.create(CRC32C, data)))
            content += data
    return blocks, bytes(content)


def test_oracle_digest_is_crc_of_filled_file(orc):
    rng = random.Random(5)
    for nb in (1, 2, 7, 40):
        blocks, content = make_file(rng, orc, nb)
        rc, ck = orc.file_digest(blocks)
        assert rc == 0
        assert ck == orc.create(CRC32C, content)
    assert orc.file_digest([]) == (0, (NONE, 0))


def test_oracle_digest_corners(orc):
    # a typed block after which a NONE block appears: combine type check (Common.h:180)
    assert orc.file_digest([(3, 3, (CRC32C, 5)), (3, 3, (NONE, 0))])[0] == 4080
    # CRC32 block with a hole: the CRC32C zero fill does not combine
    assert orc.file_digest([(1, 3, (CRC32, 5))])[0] == 4080
    # NONE blocks before the first typed one are replaced, not combined
    assert orc.file_digest([(3, 3, (NONE, 9)), (2, 2, (CRC32C, 7))]) == (0, (CRC32C, 7))
    # zero-length typed blocks are no-ops in the NONE state, type-checked after
    assert orc.file_digest([(0, 0, (CRC32, 1)), (2, 2, (CRC32C, 7))]) == (0, (CRC32C, 7))
    assert orc.file_digest([(2, 2, (CRC32C, 7)), (0, 0, (CRC32, 1))])[0] == 4080


def test_c_fold_matches_python_oracle(orc):
    """crc_oracle.c orc_file_digest_batch (the f1 CPU baseline, pthreads over files) is the same
    fold as oracle.py file_digest, both modes, status, type and value, on random corner files."""
    rng = random.Random(9)
    files = [random_corner_blocks(rng, rng.randint(0, 14)) for _ in range(400)]
    arr, off = pack_blocks(files)
    for fill_zero in (True, False):
        out = orc.file_digest_batch(arr, off, fill_zero=fill_zero, threads=3)
        for i, f in enumerate(files):
            rc, (t, v) = orc.file_digest(f, fill_zero=fill_zero)
            got = (int(out[i]["status"]), int(out[i]["type"]), int(out[i]["value"]))
            assert got == ((rc, t, v) if rc == 0 else (rc, NONE, 0)), (i, fill_zero)


# ---- a model of the kernel's summary (3fs_amd/csrc/digest_kernels.hip) ---------------------------
def _poly(t):
    return 0xEDB88320 if t == CRC32 else 0x82F63B78


def model_of_block(orc, read_len, block_len, ck):
    t, v = ck
    if t > CRC32 or read_len > block_len:
        return dict(typed=False, pre=0, nv=None, err=2)
    if read_len < block_len:
        z = block_len - read_len
        if t == NONE:
            t, v = CRC32C, orc.shift(M32, z)
        elif t == CRC32C:
            v = orc.shift(v, z)
        else:
            return dict(typed=False, pre=0, nv=None, err=1)
    if t != NONE and block_len > 0:
        return dict(typed=True, tf=t, v=v, len=block_len, pre=0, err=0)
    return dict(typed=False, pre=1 << t, nv=v if (t == NONE and block_len > 0) else None, err=0)


def model_join(orc, a, b):
    err = a["err"] | b["err"]
    if a["typed"]:
        r = dict(a)
        if b["pre"] & ~(1 << a["tf"]):
            err |= 1
        if b["typed"]:
            if b["tf"] != a["tf"]:
                err |= 1
            r["v"] = orc.shift((~a["v"]) & M32, b["len"], _poly(a["tf"])) ^ b["v"]
            r["len"] = a["len"] + b["len"]
        r["err"] = err
        return r
    if b["typed"]:
        r = dict(b)
        r["pre"] = a["pre"] | b["pre"]
        r["err"] = err
        return r
    return dict(typed=False, pre=a["pre"] | b["pre"], nv=b["nv"] if b["nv"] is not None else a["nv"], err=err)


def model_emit(s):
    if s["err"] & 2:
        return 3, (NONE, 0)
    if s["err"] & 1:
        return 4080, (NONE, 0)
    if s["typed"]:
        return 0, (s["tf"], s["v"])
    return 0, (NONE, s["nv"] if s["nv"] is not None else 0)


def model_fold(orc, blocks, cuts):
    ident = dict(typed=False, pre=0, nv=None, err=0)
    parts, prev = [], 0
    for c in list(cuts) + [len(blocks)]:
        acc = ident
        for b in blocks[prev:c]:
            acc = model_join(orc, acc, model_of_block(orc, *b))
        parts.append(acc)
        prev = c
    # pairwise tree over the partials, as the workgroup reduction does
    while len(parts) > 1:
        parts = [model_join(orc, parts[i], parts[i + 1]) if i + 1 < len(parts) else parts[i]
                 for i in range(0, len(parts), 2)]
    return model_emit(parts[0])


def random_corner_blocks(rng, n):
    out = []
    for _ in range(n):
        L = rng.choice([0, 1, 2, 3, 17, 4096])
        r = rng.choice([0, L, L, max(0, L - 1), L + 1 if rng.random() < 0.05 else L])
        t = rng.choice([NONE, CRC32C, CRC32C, CRC32C, CRC32, 3 if rng.random() < 0.02 else CRC32C])
        out.append((r, L, (t, rng.getrandbits(32))))
    return out


def test_summary_model_matches_left_fold(orc):
    rng = random.Random(11)
    for trial in range(600):
        n = rng.randint(0, 12)
        if trial % 3 == 0:  # mostly-valid files: only CRC32C and missing chunks
            blocks = [(rng.choice([0, L, L // 2]), L, (rng.choice([NONE, CRC32C, CRC32C]), rng.getrandbits(32)))
                      for L in (rng.randint(1, 300) for _ in range(n))]
            blocks = [(r if t != NONE else 0, L, (t, v if t != NONE else 0)) for r, L, (t, v) in blocks]
        else:
            blocks = random_corner_blocks(rng, n)
        cuts = sorted(rng.sample(range(n + 1), rng.randint(0, min(4, n + 1))))
        exp = orc.file_digest(blocks)
        got = model_fold(orc, blocks, cuts)
        assert got[0] == exp[0], (blocks, cuts)
        if exp[0] == 0:
            assert got == exp, (blocks, cuts)


# ---- GPU ---------------------------------------------------------------------------------------
def pack_blocks(files):
    flat = [b for f in files for b in f]
    arr = np.zeros(max(1, len(flat)), dtype=BLOCK_DT)
    for i, b in enumerate(flat):
        r, L, (t, v) = b[:3]
        arr[i] = (r, L, v, t, int(len(b) > 3 and b[3]), (0, 0))
    off = np.zeros(len(files) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(f) for f in files])
    return arr, off


def run_gpu(hf, files, fill_zero=True):
    import torch
    dev = torch.device("cuda:0")
    arr, off = pack_blocks(files)
    d_blocks = torch.from_numpy(arr.view(np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(off.view(np.int64).copy()).to(dev)
    d_out = torch.full((max(1, len(files)) * FILE_DT.itemsize,), 0xEE, dtype=torch.uint8, device=dev)
    hf._lib.file_digest_batch(d_blocks, d_off, d_out, len(files), max((len(f) for f in files), default=0),
                              stream=torch.cuda.current_stream(), fill_zero=fill_zero)
    torch.cuda.synchronize()
    return np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=FILE_DT)[:len(files)]


def check_gpu(orc, files, res, fill_zero=True):
    for i, f in enumerate(files):
        rc, (t, v) = orc.file_digest(f, fill_zero=fill_zero)
        assert int(res[i]["status"]) == rc, (i, f[:4])
        assert int(res[i]["length"]) == sum(b[1] for b in f), i
        if rc == 0:
            assert (int(res[i]["type"]), int(res[i]["value"])) == (t, v), i


@pytest.mark.gpu
def test_gpu_file_digest_real_files(hf, orc):
    rng = random.Random(21)
    files, contents = [], []
    for nb in (1, 3, 16, 255, 256, 257, 600):
        blocks, content = make_file(rng, orc, nb, max_len=700)
        files.append(blocks)
        contents.append(content)
    files.append([])
    res = run_gpu(hf, files)
    check_gpu(orc, files, res)
    for i, content in enumerate(contents):
        assert (int(res[i]["type"]), int(res[i]["value"])) == orc.create(CRC32C, content), i
    assert int(res[len(contents)]["type"]) == NONE and int(res[len(contents)]["value"]) == 0


@pytest.mark.gpu
def test_gpu_file_digest_corners(hf, orc):
    rng = random.Random(22)
    files = [random_corner_blocks(rng, rng.randint(0, 40)) for _ in range(500)]
    files += [[(0, 0, (CRC32, 1)), (2, 2, (CRC32C, 7))], [(3, 3, (NONE, 9))], [(3, 3, (NONE, 9)), (0, 4, (NONE, 0))]]
    res = run_gpu(hf, files)
    check_gpu(orc, files, res)


@pytest.mark.gpu
def test_gpu_file_digest_large_split(hf, orc):
    """Files of many blocks take the two-pass (split) path; per-block values are
    arbitrary (the fold is pure algebra), holes and missing chunks included."""
    rng = random.Random(23)
    files = []
    for nb in (5000, 40000, 150000):
        f = []
        for _ in range(nb):
            L = rng.choice([4 << 20, 4 << 20, 4 << 20, rng.randint(1, 4 << 20)])
            u = rng.random()
            if u < 0.02:
                f.append((0, L, (NONE, 0)))
            elif u < 0.05:
                f.append((rng.randint(0, L), L, (CRC32C, rng.getrandbits(32))))
            else:
                f.append((L, L, (CRC32C, rng.getrandbits(32))))
        files.append(f)
    files.append([(L, L, (CRC32C, 1)) for L in range(1, 3000)] + [(1, 1, (CRC32, 2))])  # late mismatch
    res = run_gpu(hf, files)
    check_gpu(orc, files, res)


# ---- without --fill-zero (FileWrapper.cc:134-139,153-160) ------------------------------------
def strict_files(rng, orc):
    """Files whose first failing block sits anywhere: a missing chunk (7007), a short or long
    read (33), a type mismatch before or after it (4080 only when it comes first), unknown
    types after it (3 wins: malformed input is rejected before the fold)."""
    files = []
    for k in range(400):
        n = rng.randint(0, 30)
        f = [(L, L, (CRC32C, rng.getrandbits(32))) for L in (rng.randint(0, 5000) for _ in range(n))]
        u = rng.random()
        if n and u < 0.3:
            j = rng.randrange(n)
            f[j] = (0, f[j][1], (NONE, 0), True)
        elif n and u < 0.6:
            j = rng.randrange(n)
            L = f[j][1]
            f[j] = (rng.choice([max(0, L - 1), L + 1, 0]) if L else 1, L, f[j][2])
        if n > 1 and rng.random() < 0.3:  # a CRC32 block somewhere: mismatch against CRC32C
            j = rng.randrange(n)
            f[j] = (f[j][0], f[j][1], (CRC32, 1)) + tuple(f[j][3:])
        if n and rng.random() < 0.05:
            j = rng.randrange(n)
            f[j] = (f[j][0], f[j][1], (3, 0)) + tuple(f[j][3:])
        files.append(f)
    files.append([])
    files.append([(5, 5, (CRC32C, 9)), (0, 7, (NONE, 0), True), (3, 3, (CRC32, 1))])  # 7007 before the mismatch
    files.append([(5, 5, (CRC32C, 9)), (3, 3, (CRC32, 1)), (0, 7, (NONE, 0), True)])  # 4080 before the missing
    files.append([(4, 5, (CRC32C, 9)), (5, 5, (CRC32C, 2))])  # short first block: 33
    files.append([(6, 5, (CRC32C, 9))])                      # long read: 33 (fill-zero: 3)
    return files


def test_oracle_strict_corners(orc):
    assert orc.file_digest([(5, 5, (CRC32C, 9)), (0, 7, (NONE, 0), True)], fill_zero=False)[0] == 7007
    assert orc.file_digest([(4, 5, (CRC32C, 9))], fill_zero=False)[0] == 33
    assert orc.file_digest([(6, 5, (CRC32C, 9))], fill_zero=False)[0] == 33
    assert orc.file_digest([(6, 5, (CRC32C, 9))], fill_zero=True)[0] == 3
    assert orc.file_digest([(3, 3, (CRC32, 1)), (0, 4, (NONE, 0), True)], fill_zero=False)[0] == 7007
    assert orc.file_digest([(3, 3, (CRC32C, 1)), (3, 3, (CRC32, 1)), (0, 4, (NONE, 0), True)],
                           fill_zero=False)[0] == 4080
    ok = [(3, 3, (CRC32C, 1)), (2, 2, (CRC32C, 7))]
    assert orc.file_digest(ok, fill_zero=False) == orc.file_digest(ok, fill_zero=True)
    # fill-zero: a missing chunk folds as a zero-filled read whatever checksum it carries
    assert orc.file_digest([(9, 4, (CRC32, 5), True)]) == orc.file_digest([(0, 4, (NONE, 0))])


@pytest.mark.gpu
@pytest.mark.parametrize("fill_zero", [False, True])
def test_gpu_file_digest_strict_vs_oracle(hf, orc, fill_zero):
    rng = random.Random(24 + fill_zero)
    files = strict_files(rng, orc)
    res = run_gpu(hf, files, fill_zero=fill_zero)
    check_gpu(orc, files, res, fill_zero=fill_zero)


@pytest.mark.gpu
def test_gpu_file_digest_strict_split(hf, orc):
    """Strict mode on files of many blocks (two-pass path): the first failing block lies in
    a late split, a mismatch in an earlier split comes first in another file."""
    rng = random.Random(25)
    files = []
    for nb, bad_at, mis_at in ((5000, 4000, None), (40000, 100, 39000), (40000, 39000, 100), (150000, None, None)):
        f = [(L, L, (CRC32C, rng.getrandbits(32))) for L in (rng.randint(1, 4 << 20) for _ in range(nb))]
        if bad_at is not None:
            f[bad_at] = (0, f[bad_at][1], (NONE, 0), True)
        if mis_at is not None:
            f[mis_at] = (f[mis_at][0], f[mis_at][1], (CRC32, 3))
        files.append(f)
    res = run_gpu(hf, files, fill_zero=False)
    check_gpu(orc, files, res, fill_zero=False)
    assert [int(r["status"]) for r in res] == [7007, 7007, 4080, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("fill_zero", [True, False])
@pytest.mark.parametrize("max_nb", [64, 1024, 1025])
def test_gpu_file_digest_wave_path_edges(hf, orc, fill_zero, max_nb):
    """One wave per file up to 1024 blocks (digest_kernels.hip k_digest_wave: lane runs of
    ceil(nb / 64) blocks, then the ordered register tree), the workgroup kernels above it:
    files of 0..max_nb blocks around the lane-run boundaries (63, 64, 65, 127, 128, 129, ...),
    holes, missing chunks and a first failing block anywhere, both modes, vs the oracle."""
    rng = random.Random(40 + max_nb + fill_zero)
    sizes = sorted({0, 1, 63, 64, 65, 127, 128, 129, max_nb - 1, max_nb} | {rng.randint(2, max_nb) for _ in range(12)})
    files = []
    for nb in sizes:
        for _ in range(3):
            f = [(L, L, (CRC32C, rng.getrandbits(32))) for L in (rng.choice([1, 17, 4096, 4 << 20]) for _ in range(nb))]
            for j in range(nb):
                u = rng.random()
                if u < 0.03:
                    f[j] = (0, f[j][1], (NONE, 0), True)
                elif u < 0.08:
                    f[j] = (rng.randrange(f[j][1]), f[j][1], f[j][2])
            files.append(f)
    res = run_gpu(hf, files, fill_zero=fill_zero)
    check_gpu(orc, files, res, fill_zero=fill_zero)
