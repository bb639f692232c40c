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
