"""GPU checks at the BASELINE.json sizes (2^23 -> 2^24 LDE, 2^23 x 100 Merkle).

Direct bit-exact comparison with the oracle where the oracle finishes in
seconds (a few columns), plus size-independent properties at full width:
NTT round trip, linearity of the LDE across columns, and Merkle openings that
re-hash (with the oracle's Poseidon) to the GPU root.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001


def rand_cols(torch, ncols, n, seed):
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    return torch.randint(0, 2**63 - 1, (ncols, n), dtype=torch.int64, device="cuda:0", generator=g)


@pytest.mark.parametrize("lde3", ["0", "1"])
def test_lde_2p23_vs_oracle(oracle, zkgpu, lde3, monkeypatch):
    """both LDE paths at the bench size (lde3 = the 3-pass LDE)"""
    import torch
    monkeypatch.setenv("ZKGPU_LDE3", lde3)
    n, ne, C = 1 << 23, 1 << 24, 3
    zkgpu.set_stream(torch.cuda.current_stream())
    x = rand_cols(torch, C, n, 1)
    out = torch.empty((C, ne), dtype=torch.int64, device="cuda:0")
    zkgpu.extend_pol_dev(out, ne, x, n, ne, n, C)
    torch.cuda.synchronize()
    got = zkgpu.from_device(out)
    ref = oracle.extend_pol(np.ascontiguousarray(zkgpu.from_device(x).T), ne)
    assert np.array_equal(got, ref.T)


def test_ntt_2p24_roundtrip_and_spot(oracle, zkgpu):
    import torch
    n = 1 << 24
    x = rand_cols(torch, 2, n, 2)
    y = torch.empty_like(x)
    z = torch.empty_like(x)
    zkgpu.ntt_dev(y, n, x, n, n, 2, inverse=False)
    zkgpu.ntt_dev(z, n, y, n, n, 2, inverse=True)
    torch.cuda.synchronize()
    assert torch.equal(z, x)
    # column 0 against the oracle
    ref = oracle.ntt(zkgpu.from_device(x[0]))
    assert np.array_equal(zkgpu.from_device(y[0]), ref)


def test_lde_100cols_linearity(oracle, zkgpu):
    """LDE is linear: LDE(a) + LDE(b) == LDE(a + b) column-wise, checked over
    all 100 columns at full size; column 57 also against the oracle."""
    import torch
    n, ne, C = 1 << 23, 1 << 24, 100
    a = rand_cols(torch, C, n, 3)
    out = torch.empty((C, ne), dtype=torch.int64, device="cuda:0")
    zkgpu.extend_pol_dev(out, ne, a, n, ne, n, C)
    torch.cuda.synchronize()
    # sum of columns 0 and 1 (mod p) as a new input column
    av = a[:2].cpu().numpy().view(np.uint64)
    s = ((av[0].astype(object) + av[1].astype(object)) % P).astype(np.uint64)
    ds = zkgpu.to_device(s).view(1, n)
    os_ = torch.empty((1, ne), dtype=torch.int64, device="cuda:0")
    zkgpu.extend_pol_dev(os_, ne, ds, n, ne, n, 1)
    torch.cuda.synchronize()
    o = zkgpu.from_device(out[:2])
    lin = ((o[0].astype(object) + o[1].astype(object)) % P).astype(np.uint64)
    assert np.array_equal(zkgpu.from_device(os_[0]), lin)
    ref = oracle.extend_pol(zkgpu.from_device(a[57]), ne)
    assert np.array_equal(zkgpu.from_device(out[57]), ref)


def test_merkle_2p23_x100_openings(oracle, zkgpu):
    import torch
    nrows, C = 1 << 23, 100
    src = rand_cols(torch, C, nrows, 4)
    nodes = torch.empty(zkgpu.merkle_num_elements(nrows), dtype=torch.int64, device="cuda:0")
    zkgpu.merkletree_dev(nodes, src, nrows, C, nrows)
    torch.cuda.synchronize()
    root = zkgpu.from_device(nodes[-4:])
    rng = np.random.default_rng(5)
    idx = np.concatenate([[0, nrows - 1], rng.integers(0, nrows, 30)]).astype(np.uint64)
    vals, sibs = zkgpu.merkle_open_dev(nodes, src, nrows, C, nrows, idx)
    srcT = src[:, torch.from_numpy(idx.astype(np.int64)).to("cuda:0")]
    assert np.array_equal(vals, zkgpu.from_device(srcT).T)
    for q, i in enumerate(idx):
        assert np.array_equal(oracle.merkle_root_from_proof(vals[q], sibs[q], int(i)), root)


def test_merkle_2p23_x100_tree_bit_exact(oracle, zkgpu):
    """BASELINE.md config 3 as written: the whole Poseidon Merkle tree over
    2^23 rows x 100 columns (leaves, every node level, root) equals the
    oracle's merkletree (oracle/merkle.c, OpenMP) bit for bit."""
    import os
    import torch
    nrows, C = 1 << 23, 100
    src = rand_cols(torch, C, nrows, 6)
    nodes = torch.empty(zkgpu.merkle_num_elements(nrows), dtype=torch.int64, device="cuda:0")
    zkgpu.merkletree_dev(nodes, src, nrows, C, nrows)
    torch.cuda.synchronize()
    got = zkgpu.from_device(nodes)
    rows = np.ascontiguousarray(zkgpu.from_device(src).T)  # the reference's row-major source
    del src
    oracle.lib().oc_set_num_threads(min(16, os.cpu_count() or 1))
    ref = oracle.merkletree(rows)
    assert got.shape == ref.shape
    assert np.array_equal(got[-4:], ref[-4:]), "root"
    assert np.array_equal(got, ref)
