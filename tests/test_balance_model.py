"""CPU restatement of the byte-balanced task assignment of k_crc_ranges
(3fs_amd/csrc/crc_kernels.hip: k_bal_sums + k_bal_assign),
checked against its definition: bal[k] = the first task i whose byte prefix
P_i = sum_{j<i} len_j reaches X_k = ceil(k * total / nw), bal[0] = 0,
bal[nw] = n.  The model follows the kernels' decomposition (chunks per
workgroup, runs per thread, incremental X_k) so a slip in that decomposition
shows here; the GPU parity tests cover the launch itself."""
import numpy as np
import pytest


def bal_reference(lens, nw):
    lens = np.asarray(lens, dtype=np.int64)
    n = lens.size
    total = int(lens.sum())
    bal = np.zeros(nw + 1, dtype=np.int64)
    bal[nw] = n
    if total == 0:
        for k in range(1, nw):
            bal[k] = k * n // nw
        return bal
    P = np.concatenate([[0], np.cumsum(lens)])  # P_i for i = 0..n
    for k in range(1, nw):
        X = -(-k * total // nw)
        bal[k] = int(np.searchsorted(P, X, side="left"))  # first i with P_i >= X
    return bal


def bal_model(lens, nw, nblocks, threads=256):
    """k_bal_sums / k_bal_assign as written: chunk sums, the chunk's exclusive
    base, per-thread runs with an exclusive scan, boundaries X_k in (P, P_next]."""
    lens = [int(x) for x in lens]
    n = len(lens)
    chunk = -(-n // nblocks)
    partial = [sum(lens[b * chunk:min(n, (b + 1) * chunk)]) for b in range(nblocks)]
    total = sum(partial)
    bal = [None] * (nw + 1)
    bal[0], bal[nw] = 0, n
    if total == 0:
        for k in range(1, nw):
            bal[k] = k * n // nw
        return bal
    sub = -(-chunk // threads)
    for b in range(nblocks):
        before = sum(partial[:b])
        c0, c1 = b * chunk, min(n, (b + 1) * chunk)
        runs = []
        for t in range(threads):
            r0 = min(c0 + t * sub, c1)
            r1 = min(r0 + sub, c1)
            runs.append((r0, r1, sum(lens[r0:r1])))
        acc = before
        for r0, r1, mine in runs:
            P = acc
            acc += mine
            k = P * nw // total + 1
            X = (k * total + nw - 1) // nw
            i = r0
            while i < r1 and k < nw:
                P += lens[i]
                while k < nw and X <= P:
                    assert bal[k] is None, "boundary placed twice"
                    bal[k] = i + 1
                    k += 1
                    X = (k * total + nw - 1) // nw
                i += 1
    assert all(v is not None for v in bal), "boundary never placed"
    return bal


@pytest.mark.parametrize("case", ["kv_mix", "skewed", "all_zero", "one_big", "tiny_n", "uniform"])
def test_balance_model_matches_definition(case):
    rng = np.random.default_rng(hash(case) % (1 << 32))
    nw = 4096
    if case == "kv_mix":
        lens = rng.choice([4, 8, 16, 32, 64], 200_000) * 1024
    elif case == "skewed":
        lens = np.zeros(90_000, dtype=np.int64)
        live = rng.random(lens.size) < 0.15
        lens[live] = rng.integers(1, 40_001, int(live.sum()))
        lens[30_000:30_400] = 65536
        lens[50_000] = 1 << 20
        lens[:50] = 0
        lens[-50:] = 0
    elif case == "all_zero":
        lens = np.zeros(70_000, dtype=np.int64)
    elif case == "one_big":
        lens = np.zeros(70_000, dtype=np.int64)
        lens[12345] = 1 << 30
    elif case == "tiny_n":
        nw = 64
        lens = rng.integers(0, 100, 1100)
    else:
        lens = np.full(100_000, 4096)
    nblocks = min(1024, max(1, lens.size // 1024))
    got = bal_model(lens, nw, nblocks)
    want = bal_reference(lens, nw)
    assert list(got) == list(want)
    assert all(a <= b for a, b in zip(got, got[1:]))  # contiguous, ordered runs covering every task


def test_balance_spread_beats_stride():
    """The point of the assignment: on the d5 size mix the heaviest wave carries
    close to the mean (one range over), while the static stride's heaviest wave
    is several sigma above it."""
    rng = np.random.default_rng(5)
    nw = 4096
    lens = rng.choice([4, 8, 16, 32, 64], 1_000_000).astype(np.int64) * 1024
    bal = bal_reference(lens, nw)
    P = np.concatenate([[0], np.cumsum(lens)])
    per_wave_bal = P[bal[1:]] - P[bal[:-1]]
    per_wave_stride = np.array([lens[w::nw].sum() for w in range(nw)])
    mean = lens.sum() / nw
    assert per_wave_bal.max() <= mean + lens.max()
    assert per_wave_stride.max() > mean * 1.1


# ---- byte runs (k_bal_assign with boff + byte_run in k_crc_ranges) ------------------------------
def runs_model(lens, nw, nblocks, threads=256):
    """k_bal_assign's byte-run branch as written: wave k starts at byte X_k - P_i of the range i
    with X_k in [P_i, P_i + len_i); boundaries with X_k == total point past the last range."""
    lens = [int(x) for x in lens]
    n = len(lens)
    chunk = -(-n // nblocks)
    partial = [sum(lens[b * chunk:min(n, (b + 1) * chunk)]) for b in range(nblocks)]
    total = sum(partial)
    bal, boff = [None] * (nw + 1), [None] * (nw + 1)
    bal[0], bal[nw], boff[0], boff[nw] = 0, n, 0, 0
    if total == 0:
        for k in range(1, nw):
            bal[k], boff[k] = k * n // nw, 0
        return bal, boff
    for k in range(1, nw):  # block 0: X_k == total
        if (k * total + nw - 1) // nw >= total:
            bal[k], boff[k] = n, 0
    sub = -(-chunk // threads)
    for b in range(nblocks):
        acc = sum(partial[:b])
        c0, c1 = b * chunk, min(n, (b + 1) * chunk)
        for t in range(threads):
            r0 = min(c0 + t * sub, c1)
            r1 = min(r0 + sub, c1)
            P = acc
            acc += sum(lens[r0:r1])
            k = (P - 1) * nw // total + 1 if P else 1  # first k >= 1 with X_k >= P
            X = (k * total + nw - 1) // nw
            assert X >= P and (k == 1 or ((k - 1) * total + nw - 1) // nw < P)
            for i in range(r0, r1):
                if k >= nw:
                    break
                while k < nw and X < P + lens[i]:
                    assert bal[k] is None, "boundary placed twice"
                    bal[k], boff[k] = i, X - P
                    k += 1
                    X = (k * total + nw - 1) // nw
                P += lens[i]
    assert all(v is not None for v in bal), "boundary never placed"
    return bal, boff


def run_parts(lens, bal, boff, nw):
    """byte_run's loop per wave -> covered byte parts and start terms per range."""
    n = len(lens)
    parts = [[] for _ in range(n)]
    starts = [0] * n
    for w in range(nw):
        iend, eo_last, so = bal[w + 1], boff[w + 1], boff[w]
        i = bal[w]
        while i <= iend and i < n:
            ln = int(lens[i])
            eo = eo_last if i == iend else ln
            if i == iend and eo == 0:
                break
            if ln == 0:
                starts[i] += 1
            elif so < eo:
                parts[i].append((so, eo))
                starts[i] += so == 0
            i += 1
            so = 0
    return parts, starts


@pytest.mark.parametrize("case", ["d3_pre", "tiny_total", "empties", "one_big", "all_zero", "few_blocks"])
def test_byte_runs_partition_every_range(case):
    """Every byte of every range is hashed by exactly one wave, each range's start term is added
    exactly once (empty ranges included), and the waves' shares differ by at most one byte."""
    rng = np.random.default_rng(abs(hash(case)) % (1 << 32))
    nw = 4096
    if case == "d3_pre":  # 2n jobs: payload U[64 KiB, 1 MiB], old bytes (0 for appends)
        lens = rng.integers(64 << 10, (1 << 20) + 1, 8192)
        lens[1::2] = np.where(rng.random(4096) < 0.15, 0, lens[1::2])
    elif case == "tiny_total":  # fewer bytes than waves (512 B chunks)
        lens = rng.integers(0, 60, 96)
    elif case == "empties":
        lens = np.where(rng.random(5000) < 0.7, 0, rng.integers(1, 300_000, 5000))
        lens[:7] = 0
        lens[-9:] = 0
    elif case == "one_big":
        lens = np.zeros(300, dtype=np.int64)
        lens[150] = 3 << 20
    elif case == "all_zero":
        lens = np.zeros(500, dtype=np.int64)
    else:
        lens = rng.integers(0, 2 << 20, 40)
    nblocks = min(64, max(1, lens.size // 256))
    bal, boff = runs_model(lens, nw, nblocks)
    parts, starts = run_parts(lens, bal, boff, nw)
    for i, ln in enumerate(lens):
        ps = sorted(parts[i])
        covered = 0
        for a, b in ps:
            assert a == covered, (i, ps)
            covered = b
        assert covered == int(ln), (i, ps)
        assert starts[i] == 1, (i, starts[i])
    total = int(lens.sum())
    if total:
        P = np.concatenate([[0], np.cumsum(lens)])
        pos = [int(P[bal[w]] + boff[w]) if bal[w] < len(lens) else total for w in range(nw + 1)]
        share = np.diff(pos)
        assert share.min() >= total // nw and share.max() <= -(-total // nw)
