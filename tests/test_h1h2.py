"""Plookup h1/h2 (Polinomial::calculateH1H2_opt1/_opt3, polinomial.hpp:349-583).

CPU: the C oracle vs a direct Python restatement of the reference's loop
(dict = its hash chain: key -> last row).  GPU: zkgpu_h1h2_dev vs the oracle,
bit-exact, dims 1 and 3, heavy duplicates, the missing-value error."""
import numpy as np
import pytest

P = 0xFFFFFFFF00000001


def py_h1h2(f, t):
    """polinomial.hpp:349-463 step by step (small n only)."""
    n = len(t)
    key = (lambda r: tuple(int(v) % P for v in np.atleast_1d(r)))
    last = {}
    for i in range(n):
        last[key(t[i])] = i  # the chain entry keeps the latest index (:380-383)
    counter = [1] * n
    for i in range(n):
        k = key(f[i])
        if k not in last:
            raise ValueError("Number not included: w=%d" % i)
        counter[last[k]] += 1
    h1, h2 = np.zeros_like(t), np.zeros_like(t)
    idx = 0
    for i in range(n):
        if counter[idx] == 0:
            idx += 1
        counter[idx] -= 1
        h1[i] = t[idx]
        if counter[idx] == 0:
            idx += 1
        counter[idx] -= 1
        h2[i] = t[idx]
    return h1, h2


def lookup_case(rng, n, dim, n_distinct):
    shape = (n,) if dim == 1 else (n, dim)
    vals = rng.integers(0, P, size=(n_distinct,) + shape[1:], dtype=np.uint64)
    t = vals[rng.integers(0, n_distinct, size=n)]
    f = t[rng.integers(0, n, size=n)]  # every f value is in t
    return f, t


@pytest.mark.parametrize("dim", [1, 3])
@pytest.mark.parametrize("n,distinct", [(16, 5), (256, 256), (1024, 37)])
def test_oracle_matches_reference_loop(oracle, dim, n, distinct):
    rng = np.random.default_rng(n * 7 + dim)
    f, t = lookup_case(rng, n, dim, distinct)
    h1, h2 = oracle.h1h2(f, t)
    r1, r2 = py_h1h2(f, t)
    assert np.array_equal(h1, r1) and np.array_equal(h2, r2)


def test_oracle_non_canonical_keys(oracle):
    """keys compare canonically (toU64); h1/h2 copy the table's raw words."""
    t = np.array([3, 5, 5 + P, 9], np.uint64)
    f = np.array([5, 5, 9, 3 + P], np.uint64)
    h1, h2 = oracle.h1h2(f, t)
    r1, r2 = py_h1h2(f, t)
    assert np.array_equal(h1, r1) and np.array_equal(h2, r2)
    # counts: row 0 (3) 2, row 1 (5) 1, row 2 (5+P, last 5) 3, row 3 (9) 2
    assert [int(x) for x in h1] == [3, 5, 5 + P, 9]
    assert [int(x) for x in h2] == [3, 5 + P, 5 + P, 9]


def test_oracle_missing_value(oracle):
    t = np.array([1, 2, 3, 4], np.uint64)
    f = np.array([1, 2, 7, 9], np.uint64)
    with pytest.raises(ValueError, match="w=2"):
        oracle.h1h2(f, t)


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [1, 3])
@pytest.mark.parametrize("log_n,distinct", [(10, 3), (14, 1 << 14), (16, 1000), (18, 1)])
def test_gpu_h1h2_bit_exact(oracle, zkgpu, dim, log_n, distinct):
    import torch
    rng = np.random.default_rng(log_n * 3 + dim)
    n = 1 << log_n
    f, t = lookup_case(rng, n, dim, distinct)
    r1, r2 = oracle.h1h2(f, t)
    cols = (lambda a: np.ascontiguousarray(a.reshape(n, dim).T))
    df, dt = zkgpu.to_device(cols(f)), zkgpu.to_device(cols(t))
    h1 = torch.zeros((dim, n), dtype=torch.int64, device="cuda:0")
    h2 = torch.zeros((dim, n), dtype=torch.int64, device="cuda:0")
    assert zkgpu.h1h2_dev(h1, n, h2, n, df, n, dt, n, n, dim) is None
    assert np.array_equal(zkgpu.from_device(h1).T.reshape(r1.shape), r1)
    assert np.array_equal(zkgpu.from_device(h2).T.reshape(r2.shape), r2)


@pytest.mark.gpu
def test_gpu_h1h2_non_canonical_and_missing(oracle, zkgpu):
    import torch
    n = 1 << 12
    rng = np.random.default_rng(11)
    f, t = lookup_case(rng, n, 1, 50)
    small = t < np.uint64(2**32 - 1)
    t[small] += np.uint64(P)  # same field element, non-canonical word
    r1, r2 = oracle.h1h2(f, t)
    df, dt = zkgpu.to_device(f), zkgpu.to_device(t)
    h1 = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    h2 = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    assert zkgpu.h1h2_dev(h1, n, h2, n, df, n, dt, n, n, 1) is None
    assert np.array_equal(zkgpu.from_device(h1), r1) and np.array_equal(zkgpu.from_device(h2), r2)
    f2 = f.copy()
    f2[100] = np.uint64(123456789)
    f2[3000] = np.uint64(987654321)
    if not (t == f2[100]).any() and not (t == f2[3000]).any():
        assert zkgpu.h1h2_dev(h1, n, h2, n, zkgpu.to_device(f2), n, dt, n, n, 1) == 100


@pytest.mark.gpu
def test_gpu_h1h2_dim3_shared_components(oracle, zkgpu):
    """dim 3 keys that agree in one or two components (the table must compare
    all three), non-canonical words in components 1/2, at 2^20 rows: the
    oracle's h1/h2."""
    _shared_components_case(oracle, zkgpu)


def _sharded_h1h2(zkgpu, df, dt, n, d, W):
    """calculateH1H2 through the row-sharded primitives (zkgpu_h1h2_shard_*)
    for W ranks of n / W rows, the exchanges of host/sharded_starks.hpp
    h1h2_sharded emulated by device copies in one process.  Returns (h1, h2)
    (d x n device columns) or the missing f row."""
    import torch
    nb = n // W
    dev = "cuda:0"
    recs, cnts = [], []
    for r in range(W):
        rec = torch.zeros(5 * 2 * nb, dtype=torch.int64, device=dev)
        nt, nf = zkgpu.h1h2_shard_route(rec, 2 * nb, df.data_ptr() + 8 * r * nb, n, dt.data_ptr() + 8 * r * nb, n, nb,
                                        r * nb, d, W)
        recs.append(rec)
        cnts.append((nt.astype(np.int64), nf.astype(np.int64)))
    nr = lambda s, o: int(cnts[s][0][o] + cnts[s][1][o])  # noqa: E731
    soff = [np.concatenate([[0], np.cumsum([nr(s, o) for o in range(W)])]).astype(np.int64) for s in range(W)]
    rets, roffs, misses = [], [], []
    for o in range(W):  # the owner's side of the record all-to-all
        roff = np.concatenate([[0], np.cumsum([nr(s, o) for s in range(W)])]).astype(np.int64)
        recv = torch.zeros(5 * max(int(roff[-1]), 1), dtype=torch.int64, device=dev)
        for s in range(W):
            recv[5 * roff[s]:5 * roff[s + 1]] = recs[s][5 * soff[s][o]:5 * (soff[s][o] + nr(s, o))]
        ret = torch.zeros(max(int(roff[-1]), 1), dtype=torch.int64, device=dev)
        misses.append(zkgpu.h1h2_shard_owner(ret, recv, int(roff[-1]), d))
        rets.append(ret)
        roffs.append(roff)
    if any(m is not None for m in misses):
        return min(m for m in misses if m is not None)
    tots, starts, cntl = [], [], []
    for s in range(W):  # the returns all-to-all, then the sender's counts
        ret_in = torch.zeros(max(2 * nb, 1), dtype=torch.int64, device=dev)
        for o in range(W):
            k = int(cnts[s][0][o])
            ret_in[soff[s][o]:soff[s][o] + k] = rets[o][roffs[o][s]:roffs[o][s] + k]
        start = torch.zeros(nb, dtype=torch.int32, device=dev)
        cnt = torch.zeros(nb, dtype=torch.int32, device=dev)
        tots.append(zkgpu.h1h2_shard_counts(start, cnt, recs[s], ret_in, int(soff[s][-1]), nb, s * nb))
        starts.append(start)
        cntl.append(cnt)
    assert sum(tots) == 2 * n
    off = np.concatenate([[0], np.cumsum(tots)]).astype(np.int64)
    h1 = torch.zeros((d, n), dtype=torch.int64, device=dev)
    h2 = torch.zeros((d, n), dtype=torch.int64, device=dev)
    for s in range(W):  # deal, then each piece to the rank holding its rows
        tot = tots[s]
        seg = torch.zeros(d * max(tot, 1), dtype=torch.int64, device=dev)
        zkgpu.h1h2_shard_deal(seg, max(tot, 1), dt.data_ptr() + 8 * s * nb, n, starts[s], cntl[s], nb, d)
        for e in range(W):
            a, b = max(off[s], 2 * e * nb), min(off[s] + tot, 2 * (e + 1) * nb)
            if a < b:
                zkgpu.h1h2_shard_place(h1.data_ptr() + 8 * e * nb, n, h2.data_ptr() + 8 * e * nb, n,
                                       seg.data_ptr() + 8 * int(a - off[s]), max(tot, 1), int(a), int(b - a), e * nb, d)
    return h1, h2


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_gpu_h1h2_sharded_primitives(oracle, zkgpu, world):
    """the row-sharded calculateH1H2 (zkgpu_h1h2_shard_*, the steps the
    sharded prover runs with exchanges) == the oracle: dim 3 with shared
    components and non-canonical words (2^20 rows), dim 1 with a repeated
    table value (the last row keeps the counts) and an f that is one value,
    and the smallest missing f row"""
    import torch
    rng = np.random.default_rng(world)
    n = 1 << 20
    t3, f3 = _shared_components_inputs(n)
    cols = (lambda a: np.ascontiguousarray(a.T))
    r1, r2 = oracle.h1h2(f3, t3)
    h1, h2 = _sharded_h1h2(zkgpu, zkgpu.to_device(cols(f3)), zkgpu.to_device(cols(t3)), n, 3, world)
    torch.cuda.synchronize()
    assert np.array_equal(zkgpu.from_device(h1).T, r1) and np.array_equal(zkgpu.from_device(h2).T, r2)
    n = 1 << 14
    t = rng.integers(0, P, size=n, dtype=np.uint64)
    t[7] = t[n - 5]  # a repeated table value: the later row takes the f counts
    for f in (t[rng.integers(0, n, size=n)], np.full(n, t[n - 5], np.uint64)):
        r1, r2 = oracle.h1h2(f, t)
        h1, h2 = _sharded_h1h2(zkgpu, zkgpu.to_device(f), zkgpu.to_device(t), n, 1, world)
        torch.cuda.synchronize()
        assert np.array_equal(zkgpu.from_device(h1)[0], r1) and np.array_equal(zkgpu.from_device(h2)[0], r2)
    f = t[rng.integers(0, n, size=n)]
    f[9000] = np.uint64(123456789)
    f[12000] = np.uint64(987654321)
    if not (t == f[9000]).any() and not (t == f[12000]).any():
        assert _sharded_h1h2(zkgpu, zkgpu.to_device(f), zkgpu.to_device(t), n, 1, world) == 9000


def _shared_components_inputs(n):
    rng = np.random.default_rng(20)
    base = rng.integers(0, P, size=(64, 3), dtype=np.uint64)
    vals = np.repeat(base, 16, axis=0)
    vals[:, 1] = rng.integers(0, 4, size=len(vals)).astype(np.uint64)          # few distinct second components
    vals[::2, 2] = vals[1::2, 2]                                               # pairs equal but for component 1
    vals[::3, 0] = vals[0, 0]                                                  # many share component 0
    t = vals[rng.integers(0, len(vals), size=n)]
    small = t[:, 1] < np.uint64(2**32 - 1)
    t[small, 1] += np.uint64(P)  # same element, non-canonical word
    f = t[rng.integers(0, n, size=n)] % np.uint64(P)
    return t, f


def _shared_components_case(oracle, zkgpu):
    import torch
    n = 1 << 20
    t, f = _shared_components_inputs(n)
    r1, r2 = oracle.h1h2(f, t)
    cols = (lambda a: np.ascontiguousarray(a.T))
    df, dt = zkgpu.to_device(cols(f)), zkgpu.to_device(cols(t))
    h1 = torch.zeros((3, n), dtype=torch.int64, device="cuda:0")
    h2 = torch.zeros((3, n), dtype=torch.int64, device="cuda:0")
    assert zkgpu.h1h2_dev(h1, n, h2, n, df, n, dt, n, n, 3) is None
    assert np.array_equal(zkgpu.from_device(h1).T, r1)
    assert np.array_equal(zkgpu.from_device(h2).T, r2)
