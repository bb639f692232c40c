"""GPU parity: libzkgpu (HIP, via the C-ABI) vs the CPU oracle, bit-exact.

Small and medium sizes compare against the oracle on the same seeded inputs;
the full BASELINE sizes (2^23 -> 2^24) are checked in test_gpu_large.py
through size-independent properties plus oracle spot checks.
"""
import numpy as np
import pytest

from golden_replay import check_proof

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001


def rand_gl(rng, shape, noncanon=False):
    x = (rng.integers(0, 2**63, size=shape, dtype=np.uint64) * np.uint64(2) +
         rng.integers(0, 2, size=shape, dtype=np.uint64))
    if not noncanon:
        x %= np.uint64(P)
    return x


# ------------------------------------------------------------------ NTT
@pytest.mark.parametrize("logn,ncols", [(0, 1), (1, 2), (4, 3), (8, 1), (10, 5), (12, 2), (13, 1), (14, 3),
                                        (16, 4), (17, 1), (19, 2), (20, 2)])
def test_ntt_vs_oracle(oracle, zkgpu, logn, ncols):
    rng = np.random.default_rng(100 + logn)
    x = rand_gl(rng, (1 << logn, ncols))
    for inv in (False, True):
        assert np.array_equal(zkgpu.ntt(x, inv), oracle.ntt(x, inv)), (logn, ncols, inv)


def test_ntt_noncanonical(oracle, zkgpu):
    rng = np.random.default_rng(5)
    x = rand_gl(rng, (1 << 14, 2), noncanon=True)
    assert np.array_equal(zkgpu.ntt(x), oracle.ntt(x))


@pytest.mark.parametrize("logn,blow,ncols", [(0, 1, 1), (3, 1, 2), (10, 1, 3), (12, 1, 4), (13, 1, 2),
                                             (14, 2, 3), (16, 1, 8), (17, 1, 2), (18, 1, 2), (19, 1, 3),
                                             (20, 1, 2), (21, 1, 1), (22, 1, 1)])
@pytest.mark.parametrize("lde3", ["0", "1"])
def test_extend_pol_vs_oracle(oracle, zkgpu, logn, blow, ncols, lde3, monkeypatch):
    """both LDE paths: the 6-pass NTT chain and (2^18..2^24, blowup 1) the
    3-pass LDE of ntt.hip (ZKGPU_LDE3=1)"""
    monkeypatch.setenv("ZKGPU_LDE3", lde3)
    rng = np.random.default_rng(200 + logn)
    x = rand_gl(rng, (1 << logn, ncols))
    ne = 1 << (logn + blow)
    assert np.array_equal(zkgpu.extend_pol(x, ne), oracle.extend_pol(x, ne))


@pytest.mark.parametrize("logn,ncols,lde3", [(15, 5, "0"), (18, 3, "1"), (20, 7, "1"), (20, 2, "0")])
def test_extend_pol_dev_column_major(oracle, zkgpu, logn, ncols, lde3, monkeypatch):
    """Device-resident SoA path with padded leading dimensions (lde3: the
    3-pass LDE of ntt.hip)."""
    import torch
    monkeypatch.setenv("ZKGPU_LDE3", lde3)
    rng = np.random.default_rng(9 + logn)
    n, ne = 1 << logn, 1 << (logn + 1)
    x = rand_gl(rng, (n, ncols))
    ld_in, ld_out = n + 64, ne + 128
    cols = np.zeros((ncols, ld_in), np.uint64)
    cols[:, :n] = x.T
    din = zkgpu.to_device(cols)
    dout = torch.zeros((ncols, ld_out), dtype=torch.int64, device="cuda:0")
    zkgpu.set_stream(torch.cuda.current_stream())
    zkgpu.extend_pol_dev(dout, ld_out, din, ld_in, ne, n, ncols)
    torch.cuda.synchronize()
    got = zkgpu.from_device(dout)[:, :ne].T
    assert np.array_equal(got, oracle.extend_pol(x, ne))


# ------------------------------------------------------------------ Poseidon
def test_poseidon_vs_oracle(oracle, zkgpu):
    rng = np.random.default_rng(11)
    for i in range(20):
        x = rand_gl(rng, 12, noncanon=(i % 3 == 0))
        assert np.array_equal(zkgpu.poseidon_full(x), oracle.poseidon_full(x))
        assert np.array_equal(zkgpu.poseidon_hash(x), oracle.poseidon_hash(x))
    for x in (np.zeros(12, np.uint64), np.full(12, P - 1, np.uint64)):
        assert np.array_equal(zkgpu.poseidon_full(x), oracle.poseidon_full(x))


def test_poseidon_batch_dev(oracle, zkgpu):
    import torch
    rng = np.random.default_rng(12)
    n = 10000
    x = rand_gl(rng, (n, 12))
    din = zkgpu.to_device(x)
    dout = torch.zeros((n, 12), dtype=torch.int64, device="cuda:0")
    zkgpu.poseidon_batch_dev(dout, din, n, True)
    torch.cuda.synchronize()
    got = zkgpu.from_device(dout)
    for i in (0, 1, 4097, n - 1):
        assert np.array_equal(got[i], oracle.poseidon_full(x[i]))


@pytest.mark.parametrize("size", [0, 1, 3, 4, 5, 8, 9, 16, 17, 52, 100])
def test_linear_hash_vs_oracle(oracle, zkgpu, size):
    rng = np.random.default_rng(300 + size)
    x = rand_gl(rng, size)
    assert np.array_equal(zkgpu.linear_hash(x), oracle.linear_hash(x))


# ------------------------------------------------------------------ Merkle
@pytest.mark.parametrize("nrows,ncols", [(1, 5), (2, 3), (256, 0), (1024, 13), (4096, 100), (2048, 4), (8192, 9)])
def test_merkletree_vs_oracle(oracle, zkgpu, nrows, ncols):
    rng = np.random.default_rng(nrows + ncols)
    src = rand_gl(rng, (nrows, ncols))
    assert np.array_equal(zkgpu.merkletree(src), oracle.merkletree(src))


def test_merkletree_dev_and_openings(oracle, zkgpu):
    import torch
    rng = np.random.default_rng(21)
    nrows, ncols = 1 << 12, 21
    src = rand_gl(rng, (nrows, ncols))
    dsrc = zkgpu.to_device(np.ascontiguousarray(src.T))
    nodes = torch.zeros(zkgpu.merkle_num_elements(nrows), dtype=torch.int64, device="cuda:0")
    zkgpu.merkletree_dev(nodes, dsrc, nrows, ncols, nrows)
    torch.cuda.synchronize()
    ref_nodes = oracle.merkletree(src)
    assert np.array_equal(zkgpu.from_device(nodes), ref_nodes)
    idx = np.array([0, 1, 7, 2048, nrows - 1], np.uint64)
    vals, sibs = zkgpu.merkle_open_dev(nodes, dsrc, nrows, ncols, nrows, idx)
    for q, i in enumerate(idx):
        v, s = oracle.merkle_group_proof(ref_nodes, src, int(i))
        assert np.array_equal(vals[q], v)
        assert np.array_equal(sibs[q], s)


def test_merkletree_rows_dev(oracle, zkgpu):
    import torch
    rng = np.random.default_rng(22)
    nrows, ncols = 1 << 10, 48
    src = rand_gl(rng, (nrows, ncols))
    nodes = torch.zeros(zkgpu.merkle_num_elements(nrows), dtype=torch.int64, device="cuda:0")
    zkgpu.merkletree_rows_dev(nodes, zkgpu.to_device(src), ncols, nrows)
    torch.cuda.synchronize()
    assert np.array_equal(zkgpu.from_device(nodes), oracle.merkletree(src))


def test_merkle_open_many_vs_oracle(oracle, zkgpu):
    """The query phase's one-round-trip openings (zkgpu_gl_merkle_open_many):
    a column-major tree, a row-major tree, an empty request and a width-0
    tree, each equal to the oracle's getGroupProof; a bad index anywhere fails
    the whole call before anything is queued."""
    import torch
    rng = np.random.default_rng(23)
    trees = []
    for nrows, ncols, rows in [(1 << 11, 13, False), (1 << 9, 24, True), (1 << 10, 0, False)]:
        src = rand_gl(rng, (nrows, ncols))
        nodes = torch.zeros(zkgpu.merkle_num_elements(nrows), dtype=torch.int64, device="cuda:0")
        dsrc = zkgpu.to_device(src if rows else np.ascontiguousarray(src.T)) if ncols else nodes
        if rows:
            zkgpu.merkletree_rows_dev(nodes, dsrc, ncols, nrows)
        else:
            zkgpu.merkletree_dev(nodes, dsrc, nrows, ncols, nrows)
        torch.cuda.synchronize()
        trees.append((src, nodes, dsrc, nrows, ncols, rows))
    reqs, idxs = [], []
    for k, (src, nodes, dsrc, nrows, ncols, rows) in enumerate(trees):
        idx = rng.integers(0, nrows, 9 + k, dtype=np.uint64)
        idx[0], idx[-1] = 0, nrows - 1
        idxs.append(idx)
        reqs.append((nodes, dsrc, nrows, ncols, nrows, idx, rows))
    reqs.insert(1, (trees[0][1], trees[0][2], trees[0][3], trees[0][4], trees[0][3], np.zeros(0, np.uint64), False))
    got = zkgpu.merkle_open_many(reqs)
    del got[1]
    for (src, nodes, _, nrows, ncols, _), idx, (vals, sibs) in zip(trees, idxs, got):
        ref_nodes = oracle.merkletree(src)
        for q, i in enumerate(idx):
            v, s = oracle.merkle_group_proof(ref_nodes, src, int(i))
            assert np.array_equal(vals[q], v)
            assert np.array_equal(sibs[q], s)
    bad = list(reqs)
    bad[-1] = bad[-1][:5] + (np.array([0, bad[-1][4]], np.uint64),) + bad[-1][6:]
    with pytest.raises(zkgpu.ZkgpuError, match="index"):
        zkgpu.merkle_open_many(bad)
    bad[-1] = bad[-1][:4] + (bad[-1][4] - 1, np.zeros(1, np.uint64)) + bad[-1][6:]
    with pytest.raises(zkgpu.ZkgpuError, match="power of two"):
        zkgpu.merkle_open_many(bad)
    assert zkgpu.merkle_open_many([]) == []


def test_stream_marks(zkgpu):
    """zkgpu_mark / zkgpu_mark_elapsed (the host prover's stage timers): the
    time between two marks around queued work, and the argument checks."""
    import ctypes
    import torch
    L = zkgpu.lib()
    nodes = torch.zeros(zkgpu.merkle_num_elements(1 << 12), dtype=torch.int64, device="cuda:0")
    src = zkgpu.to_device(np.ascontiguousarray(rand_gl(np.random.default_rng(5), (1 << 12, 9)).T))
    assert L.zkgpu_mark(200) == 0
    zkgpu.merkletree_dev(nodes, src, 1 << 12, 9, 1 << 12)
    assert L.zkgpu_mark(201) == 0
    ms = ctypes.c_double(-1.0)
    assert L.zkgpu_mark_elapsed(200, 201, ctypes.byref(ms)) == 0
    assert 0.0 < ms.value < 1000.0
    assert L.zkgpu_mark(256) != 0  # (ZKGPU_MARKS slots)
    assert L.zkgpu_mark_elapsed(200, 255, ctypes.byref(ms)) != 0  # never recorded


# ------------------------------------------------------------------ FRI
@pytest.mark.parametrize("pol_bits,out_bits", [(6, 2), (10, 6), (12, 9), (16, 12), (20, 16), (11, 11), (13, 8)])
def test_fri_fold_vs_oracle(oracle, zkgpu, pol_bits, out_bits):
    import torch
    rng = np.random.default_rng(pol_bits * 31 + out_bits)
    pol = rand_gl(rng, 3 << pol_bits)
    sx = rand_gl(rng, 3)
    sinv = oracle.gl_pow(oracle.gl_inv(7), 1 << (pol_bits % 5))
    dpol = zkgpu.to_device(pol)
    dout = torch.zeros(3 << out_bits, dtype=torch.int64, device="cuda:0")
    zkgpu.fri_fold_dev(dout, dpol, pol_bits, out_bits, sx, sinv)
    torch.cuda.synchronize()
    assert np.array_equal(zkgpu.from_device(dout), oracle.fri_fold(pol, pol_bits, out_bits, sx, sinv))


@pytest.mark.parametrize("pol_bits,out_bits,g0,ng", [(12, 8, 64, 64), (16, 12, 0, 512), (11, 7, 96, 32), (10, 5, 31, 1)])
def test_fri_fold_rows_vs_oracle(oracle, zkgpu, pol_bits, out_bits, g0, ng):
    """zkgpu_fri_fold_rows_dev (the sharded prover's first fold): groups
    [g0, g0 + ng) from their getTransposed rows == those outputs of the
    oracle's whole fold"""
    import torch
    rng = np.random.default_rng(pol_bits * 7 + g0)
    pol = rand_gl(rng, 3 << pol_bits)
    sx = rand_gl(rng, 3)
    sinv = oracle.gl_pow(oracle.gl_inv(7), 1 << (pol_bits % 5))
    kk = 1 << (pol_bits - out_bits)
    rows = oracle.fri_get_transposed(pol, out_bits).reshape(1 << out_bits, 3 * kk)[g0:g0 + ng]
    dout = torch.zeros(3 * ng, dtype=torch.int64, device="cuda:0")
    zkgpu.fri_fold_rows_dev(dout, zkgpu.to_device(np.ascontiguousarray(rows)), g0, ng, pol_bits, out_bits, sx, sinv)
    torch.cuda.synchronize()
    want = oracle.fri_fold(pol, pol_bits, out_bits, sx, sinv).reshape(-1, 3)[g0:g0 + ng]
    assert np.array_equal(zkgpu.from_device(dout).reshape(-1, 3), want)


def test_fri_transpose(oracle, zkgpu):
    import torch
    rng = np.random.default_rng(23)
    pol = rand_gl(rng, 3 << 12)
    daux = torch.zeros(3 << 12, dtype=torch.int64, device="cuda:0")
    zkgpu.fri_transpose_dev(daux, zkgpu.to_device(pol), 1 << 12, 8)
    torch.cuda.synchronize()
    assert np.array_equal(zkgpu.from_device(daux), oracle.fri_get_transposed(pol, 8))


# ------------------------------------------------------------------ golden, through the GPU
@pytest.mark.parametrize("name", ["recursive1.zkin.proof_0.json", "recursive2.zkin.proof_01.json"])
def test_golden_replay_on_gpu(oracle, zkgpu, name):
    """The reference's own proofs re-derived with GPU Poseidon/linear-hash and
    the GPU fold kernel (transcript order and query indices from the oracle)."""
    import torch

    def root_from_proof(vals, sibs, idx):
        cur = zkgpu.linear_hash(vals)
        for s in np.asarray(sibs, np.uint64).reshape(-1, 4):
            pair = np.concatenate([s, cur]) if idx & 1 else np.concatenate([cur, s])
            cur = zkgpu.poseidon_hash(np.concatenate([pair, np.zeros(4, np.uint64)]))
            idx >>= 1
        return cur

    cache = {}

    def fold_group(vals, g, pol_bits, sx, sinv):
        nx = vals.size // 3
        out_bits = pol_bits - (nx.bit_length() - 1)
        key = (pol_bits, out_bits)
        if key not in cache:
            cache[key] = (torch.zeros(3 << pol_bits, dtype=torch.int64, device="cuda:0"),
                          torch.zeros(3 << out_bits, dtype=torch.int64, device="cuda:0"))
        dpol, dout = cache[key]
        dpol.zero_()
        v = torch.from_numpy(np.ascontiguousarray(vals, np.uint64).view(np.int64)).to("cuda:0")
        idx = torch.tensor([(j << out_bits) + g for j in range(nx)], device="cuda:0")
        dpol.view(-1, 3)[idx] = v.view(-1, 3)
        zkgpu.fri_fold_dev(dout, dpol, pol_bits, out_bits, sx, sinv)
        torch.cuda.synchronize()
        return zkgpu.from_device(dout[3 * g:3 * g + 3])

    bad, _ = check_proof(oracle, name, root_from_proof=root_from_proof, fold_group=fold_group)
    assert bad["s0"] == 0 and bad["fri_tree"] == 0 and bad["fold"] == 0 and bad["final"] == 0


# ------------------------------------------------------------------ arithmetic core
def _adversarial(rng, n):
    """u64 values concentrated on the reduction edges (>= p, near 2^64, 2^32 boundaries)."""
    special = [0, 1, 2, P - 2, P - 1, P, P + 1, P + 2**31, 2**64 - 2, 2**64 - 1, 2**32 - 1, 2**32, 2**32 + 1,
               2**63, 2**63 - 1, 2**64 - 2**32, 2**64 - 2**32 - 1, 2**48, 2**96 % P, 0xFFFFFFFF00000000]
    vals = list(special) + [int(v) for v in rng.integers(0, 2**64 - 1, size=n - len(special), dtype=np.uint64,
                                                            endpoint=True)]
    # half of the random ones pushed into [p, 2^64)
    out = []
    for i, v in enumerate(vals):
        if i >= len(special) and i % 2:
            v = P + v % (2**64 - P)
        out.append(v)
    return np.array(out, dtype=np.uint64)


@pytest.mark.parametrize("op", list(range(9)))
def test_field_core_adversarial(zkgpu, op):
    import torch
    rng = np.random.default_rng(op)
    n = 4096
    a = _adversarial(rng, n)
    b = _adversarial(rng, n)[::-1].copy()
    # all pairs of the special values too
    sp = a[:20]
    a = np.concatenate([a, np.repeat(sp, 20)])
    b = np.concatenate([b, np.tile(sp, 20)])
    n = a.size
    out = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    zkgpu.field_selftest_dev(out, zkgpu.to_device(a), zkgpu.to_device(b), n, op)
    torch.cuda.synchronize()
    got = zkgpu.from_device(out)
    A = [int(x) for x in a]
    B = [int(x) for x in b]
    f = {0: lambda x, y: x + y, 1: lambda x, y: x - y, 2: lambda x, y: x * y, 3: lambda x, y: -x,
         4: lambda x, y: x << 12, 5: lambda x, y: x << 48, 6: lambda x, y: x << 84, 7: lambda x, y: x << 100,
         8: lambda x, y: pow(x, 7, P)}[op]
    exp = np.array([f(x, y) % P for x, y in zip(A, B)], dtype=np.uint64)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(hex(A[i]), hex(B[i]), hex(int(got[i])), hex(int(exp[i]))) for i in bad[:5]]


def test_field_cubic_adversarial(oracle, zkgpu):
    import torch
    rng = np.random.default_rng(99)
    n = 2000
    a = _adversarial(rng, 3 * n)
    b = _adversarial(rng, 3 * n)[::-1].copy()
    out = torch.zeros(3 * n, dtype=torch.int64, device="cuda:0")
    zkgpu.field_selftest_dev(out, zkgpu.to_device(a), zkgpu.to_device(b), n, 9)
    torch.cuda.synchronize()
    got = zkgpu.from_device(out)
    for i in range(n):
        assert np.array_equal(got[3 * i:3 * i + 3], oracle.gl3_mul(a[3 * i:3 * i + 3], b[3 * i:3 * i + 3])), i
