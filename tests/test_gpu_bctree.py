"""GPU parity for the constant-tree builder (tools/starkpil/bctree) and the
executor hand-off loader, through the C-ABI, bit-exact against the oracle.

The const-tree file layout follows build_const_tree.cpp:566-603:
[nPols, nExt, LDE row-major (nExt x nPols), Merkle nodes], verkey constRoot =
last 4 elements.  The oracle composes its extendPol restatement (pinned by the
golden proofs' shift/omega conventions) with its merkletree (pinned by the
golden openings).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001


def rand_gl(rng, shape):
    return rng.integers(0, 2**63, size=shape, dtype=np.uint64) % np.uint64(P)


@pytest.mark.parametrize("n_bits,blow,n_pols", [(4, 1, 3), (10, 1, 7), (12, 2, 5), (14, 1, 20), (10, 1, 0),
                                                (13, 1, 1)])
def test_build_const_tree_vs_oracle(oracle, zkgpu, n_bits, blow, n_pols):
    rng = np.random.default_rng(700 + n_bits + n_pols)
    n, n_ext = 1 << n_bits, 1 << (n_bits + blow)
    pols = rand_gl(rng, (n, n_pols))
    tree = zkgpu.build_const_tree(pols, n_bits + blow)
    assert tree.size == 2 + n_pols * n_ext + 8 * n_ext - 4
    assert int(tree[0]) == n_pols and int(tree[1]) == n_ext
    if n_pols:
        lde = oracle.extend_pol(pols, n_ext)
        assert np.array_equal(tree[2:2 + n_pols * n_ext].reshape(n_ext, n_pols), lde)
    else:
        lde = np.zeros((n_ext, 0), np.uint64)
    nodes = oracle.merkletree(lde)
    assert np.array_equal(tree[2 + n_pols * n_ext:], nodes)


def test_const_tree_root_matches_merkletree_of_lde(zkgpu):
    """The verkey (last 4) equals the root of the GPU merkletree over the GPU LDE."""
    rng = np.random.default_rng(11)
    pols = rand_gl(rng, (1 << 12, 9))
    tree = zkgpu.build_const_tree(pols, 13)
    lde = zkgpu.extend_pol(pols, 1 << 13)
    assert np.array_equal(tree[-4:], zkgpu.merkletree(lde)[-4:])


@pytest.mark.parametrize("nrows,ncols,block,register", [(1000, 13, 96, False), (4096, 751, 0, False),
                                                         (777, 5, 1000, True), (64, 1, 7, True)])
def test_load_rows_dev(zkgpu, nrows, ncols, block, register):
    import torch
    rng = np.random.default_rng(nrows + ncols)
    rows = rng.integers(0, 2**64 - 1, size=(nrows, ncols), dtype=np.uint64)
    ld = nrows + 32
    cols = torch.zeros(ncols * ld, dtype=torch.int64, device="cuda:0")
    zkgpu.load_rows_dev(cols, ld, rows, block_rows=block, register_host=register)
    torch.cuda.synchronize()
    got = zkgpu.from_device(cols).reshape(ncols, ld)[:, :nrows]
    assert np.array_equal(got, rows.T)


@pytest.mark.parametrize("nrows,ncols,block", [(1000, 13, 96), (4096, 751, 0), (64, 1, 7)])
def test_load_rows_async(zkgpu, nrows, ncols, block):
    """The background loader (zkgpu_load_rows_async on the library's loader
    thread and streams) lands the same columns as the synchronous one, while
    kernels on the library stream run beside it; a too-small stage is refused."""
    import torch
    rng = np.random.default_rng(7 * nrows + ncols)
    rows = rng.integers(0, 2**64 - 1, size=(nrows, ncols), dtype=np.uint64)
    ld = nrows + 8
    cols = torch.zeros(ncols * ld, dtype=torch.int64, device="cuda:0")
    stage_bytes = zkgpu.load_rows_stage_bytes(nrows, ncols, block)
    stage = torch.empty((stage_bytes + 7) // 8, dtype=torch.int64, device="cuda:0")
    job = zkgpu.load_rows_async(cols, ld, rows, stage, block_rows=block)
    busy = zkgpu.merkletree(rng.integers(0, 2**63, size=(1 << 12, 8), dtype=np.uint64))  # library-stream work meanwhile
    job.wait()
    torch.cuda.synchronize()
    got = zkgpu.from_device(cols).reshape(ncols, ld)[:, :nrows]
    assert np.array_equal(got, rows.T) and busy.size
    small = torch.empty(max(1, stage_bytes // 16), dtype=torch.int64, device="cuda:0")
    with pytest.raises(zkgpu.ZkgpuError, match="stage"):
        zkgpu.load_rows_async(cols, ld, rows, small, block_rows=block)
