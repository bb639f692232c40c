"""Checks of the CPU oracle itself (field, NTT/LDE, Merkle, FRI helpers).

The big NTT/LDE has no reference data at scale; it is pinned here by the
O(n^2) definition at small n, by algebraic properties (round trip, coset
evaluation) and, in test_golden_proofs.py, by the reference's FRI folds.
"""
import numpy as np
import pytest

P = 0xFFFFFFFF00000001


def rand_gl(rng, shape):
    return (rng.integers(0, 2**63, size=shape, dtype=np.uint64) * np.uint64(2) +
            rng.integers(0, 2, size=shape, dtype=np.uint64)) % np.uint64(P)


def test_roots_of_unity(oracle):
    # W[1..8]
    expect = [P - 1, 2**48, 2**24, 4096, 64, 8, 2198989700608, 4404853092538523347]
    assert [oracle.gl_w(n) for n in range(1, 9)] == expect
    assert oracle.gl_w(0) == 1
    for n in (16, 23, 24, 32):
        w = oracle.gl_w(n)
        assert oracle.gl_pow(w, 1 << n) == 1
        assert oracle.gl_pow(w, 1 << (n - 1)) == P - 1


def test_field_ops_bigint(oracle):
    rng = np.random.default_rng(1)
    xs = [int(v) for v in rand_gl(rng, 200)] + [0, 1, P - 1, P - 2, 2**32, 2**64 - 1, P, P + 5]
    for i in range(len(xs) - 1):
        a, b = xs[i], xs[i + 1]
        assert oracle.gl_mul(a, b) == (a * b) % P
        assert oracle.gl_add(a, b) == (a + b) % P
        assert oracle.gl_sub(a, b) == (a - b) % P
        if a % P:
            assert (oracle.gl_inv(a) * a) % P == 1


def _poly3_mul(a, b):
    # reduce modulo x^3 - x - 1
    c = [0] * 5
    for i in range(3):
        for j in range(3):
            c[i + j] += a[i] * b[j]
    c[2] += c[4]; c[1] += c[4]  # x^4 = x^2 + x
    c[1] += c[3]; c[0] += c[3]  # x^3 = x + 1
    return [v % P for v in c[:3]]


def test_cubic_extension(oracle):
    rng = np.random.default_rng(2)
    for _ in range(50):
        a = [int(v) for v in rand_gl(rng, 3)]
        b = [int(v) for v in rand_gl(rng, 3)]
        assert [int(v) for v in oracle.gl3_mul(a, b)] == _poly3_mul(a, b)
        inv = oracle.gl3_inv(a)
        assert [int(v) for v in oracle.gl3_mul(a, inv)] == [1, 0, 0]


@pytest.mark.parametrize("logn,ncols", [(0, 1), (1, 3), (4, 3), (6, 1), (9, 5)])
def test_ntt_vs_naive(oracle, logn, ncols):
    rng = np.random.default_rng(logn)
    x = rand_gl(rng, (1 << logn, ncols))
    for inv in (False, True):
        assert np.array_equal(oracle.ntt(x, inv), oracle.dft_naive(x, inv))


def test_ntt_large_roundtrip(oracle):
    rng = np.random.default_rng(7)
    x = rand_gl(rng, (1 << 16, 4))
    y = oracle.ntt(x)
    assert np.array_equal(oracle.ntt(y, True), x)
    # spot-check output entries against the definition
    w = oracle.gl_w(16)
    for k in (0, 1, 12345, (1 << 16) - 1):
        acc = 0
        wk = pow(w, k, P)
        for j in range(1 << 16):
            acc = (acc + int(x[j, 2]) * pow(wk, j, P)) % P
        assert int(y[k, 2]) == acc


def test_ntt_noncanonical_inputs(oracle):
    x = np.array([P, P + 1, 2**64 - 1, 3], np.uint64)
    canon = np.array([0, 1, (2**64 - 1) % P, 3], np.uint64)
    assert np.array_equal(oracle.ntt(x), oracle.ntt(canon))


@pytest.mark.parametrize("logn,blow,ncols", [(3, 1, 2), (5, 1, 3), (5, 2, 1), (8, 1, 4)])
def test_extend_pol_coset(oracle, logn, blow, ncols):
    """out[i] = P(7 * w_next^i) with P interpolating the input on <w_n>."""
    rng = np.random.default_rng(logn * 10 + blow)
    n, ne = 1 << logn, 1 << (logn + blow)
    x = rand_gl(rng, (n, ncols))
    out = oracle.extend_pol(x, ne)
    coef = oracle.dft_naive(x, True)
    we = oracle.gl_w(logn + blow)
    for i in range(ne):
        pt = 7 * pow(we, i, P) % P
        for c in range(ncols):
            acc = 0
            for k in range(n - 1, -1, -1):
                acc = (acc * pt + int(coef[k, c])) % P
            assert int(out[i, c]) == acc


def test_merkle_group_proofs(oracle):
    rng = np.random.default_rng(3)
    for nrows, ncols in [(1, 5), (2, 4), (16, 9), (64, 13), (32, 0)]:
        src = rand_gl(rng, (nrows, ncols))
        nodes = oracle.merkletree(src)
        assert nodes.size == 4 * nrows + 4 * (nrows - 1)
        root = oracle.merkle_root(nodes)
        for idx in range(nrows):
            vals, sib = oracle.merkle_group_proof(nodes, src, idx)
            assert sib.shape[0] == (nrows.bit_length() - 1)
            assert np.array_equal(oracle.merkle_root_from_proof(vals, sib, idx), root)


def test_linear_hash_short(oracle):
    assert np.array_equal(oracle.linear_hash([5, 6]), np.array([5, 6, 0, 0], np.uint64))
    assert np.array_equal(oracle.linear_hash([]), np.zeros(4, np.uint64))


def test_fri_fold_full_vs_group(oracle):
    rng = np.random.default_rng(5)
    pol_bits, out_bits = 10, 6
    pol = rand_gl(rng, 3 << pol_bits)
    sx = rand_gl(rng, 3)
    sinv = oracle.gl_inv(7)
    full = oracle.fri_fold(pol, pol_bits, out_bits, sx, sinv)
    for g in (0, 1, 37, 63):
        vals = np.concatenate([pol[3 * (j * 64 + g):3 * (j * 64 + g) + 3] for j in range(16)])
        assert np.array_equal(oracle.fri_fold_group(vals, g, pol_bits, sx, sinv), full[3 * g:3 * g + 3])


def test_fri_fold_low_degree(oracle):
    """Folding the coset LDE of a degree < d polynomial yields a degree < d/r one."""
    rng = np.random.default_rng(6)
    n_bits, blow, red = 6, 2, 2
    coef = np.zeros((1 << (n_bits + blow), 3), np.uint64)
    coef[: 1 << n_bits] = rand_gl(rng, (1 << n_bits, 3))
    # evaluations on the coset 7*<w>
    ev = oracle.extend_pol(oracle.ntt(coef[: 1 << n_bits]), 1 << (n_bits + blow))
    sx = rand_gl(rng, 3)
    out = oracle.fri_fold(ev, n_bits + blow, n_bits + blow - red, sx, oracle.gl_inv(7))
    # out lives on the coset 7^(2^red) * <w'>: interpolate and check high coefs vanish
    shift = pow(7, 1 << red, P)
    m = 1 << (n_bits + blow - red)
    c = oracle.ntt(out.reshape(m, 3), True)
    sinv = pow(shift, P - 2, P)
    c = np.array([[int(c[i, k]) * pow(sinv, i, P) % P for k in range(3)] for i in range(m)], dtype=object)
    assert all(int(v) == 0 for v in c[1 << (n_bits - red):].ravel())


def test_batch_inverse3(oracle):
    rng = np.random.default_rng(8)
    x = rand_gl(rng, 3 * 33)
    inv = oracle.batch_inverse3(x)
    for i in range(33):
        assert np.array_equal(inv[3 * i:3 * i + 3], oracle.gl3_inv(x[3 * i:3 * i + 3]))


def test_config1_ntt_2p20_roundtrip(oracle):
    """BASELINE configs[0]: the 2^20-point forward + inverse NTT on the CPU is
    the identity (NTT_Goldilocks::NTT / INTT, starks.cpp:262,285); plus two
    outputs against the DFT definition (Horner over the 2^20 inputs)."""
    import time
    rng = np.random.default_rng(20)
    n = 1 << 20
    x = rand_gl(rng, (n, 2))
    t0 = time.perf_counter()
    y = oracle.ntt(x)
    z = oracle.ntt(y, True)
    dt = time.perf_counter() - t0
    assert np.array_equal(z, x)
    w = oracle.gl_w(20)
    for k in (1, n - 3):
        wk = pow(w, k, P)
        acc = 0
        for v in x[::-1, 1].tolist():  # Horner: sum_j x_j wk^j
            acc = (acc * wk + v) % P
        assert int(y[k, 1]) == acc
    print("config 1: 2^20 x 2 forward + inverse NTT on the CPU oracle in %.3f s" % dt)
