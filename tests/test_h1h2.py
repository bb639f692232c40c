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
@pytest.mark.parametrize("sort_path", [False, True])
def test_gpu_h1h2_dim3_shared_components(oracle, zkgpu, sort_path, monkeypatch):
    """dim 3 keys that agree in one or two components (the table must compare
    all three), non-canonical words in components 1/2, at 2^20 rows; both the
    hash path (default) and the sort path (ZKGPU_H1H2_SORT=1, read once per
    process: run in a child) give the oracle's h1/h2."""
    import subprocess
    import sys
    if sort_path:
        code = ("import sys; sys.path[:0] = %r\n"
                "import test_h1h2 as T\n"
                "from oracle import oracle as oc\nimport zkgpu\noc.lib()\nzkgpu.init()\n"
                "T._shared_components_case(oc, zkgpu)\n") % ([ROOT_DIR, ROOT_DIR + "/zkevm-prover_amd",
                                                               ROOT_DIR + "/tests"],)
        env = dict(__import__("os").environ, ZKGPU_H1H2_SORT="1")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
    else:
        _shared_components_case(oracle, zkgpu)


ROOT_DIR = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


def _shared_components_case(oracle, zkgpu):
    import torch
    n = 1 << 20
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
    r1, r2 = oracle.h1h2(f, t)
    cols = (lambda a: np.ascontiguousarray(a.T))
    df, dt = zkgpu.to_device(cols(f)), zkgpu.to_device(cols(t))
    h1 = torch.zeros((3, n), dtype=torch.int64, device="cuda:0")
    h2 = torch.zeros((3, n), dtype=torch.int64, device="cuda:0")
    assert zkgpu.h1h2_dev(h1, n, h2, n, df, n, dt, n, n, 3) is None
    assert np.array_equal(zkgpu.from_device(h1).T, r1)
    assert np.array_equal(zkgpu.from_device(h2).T, r2)
