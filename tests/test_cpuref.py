"""bench.py's CPU baseline (cpuref/: the reference's AVX2 + OpenMP path for
the proof's bulk kernels, restated) computes exactly what the oracle computes
-- so its timing is of the same proof.  CPU only."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def cr():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpuref"))
    import cpuref
    cpuref.lib()
    return cpuref


@pytest.mark.parametrize("nrows,ncols", [(1, 3), (2, 4), (4, 5), (8, 9), (64, 100), (1 << 10, 17), (1 << 11, 751)])
def test_merkletree_equals_oracle(oracle, cr, nrows, ncols):
    x = np.random.default_rng(nrows + ncols).integers(0, 2**64, size=(nrows, ncols), dtype=np.uint64)
    assert np.array_equal(cr.merkletree(x), oracle.merkletree(x))


@pytest.mark.parametrize("n,ne,nc", [(1, 2, 3), (8, 16, 5), (1 << 10, 1 << 11, 7), (1 << 12, 1 << 14, 13),
                                     (1 << 13, 1 << 14, 100)])
def test_extend_pol_and_ntt_equal_oracle(oracle, cr, n, ne, nc):
    x = np.random.default_rng(n + nc).integers(0, 2**64, size=(n, nc), dtype=np.uint64)
    assert np.array_equal(cr.extend_pol(x, ne), oracle.extend_pol(x, ne))
    for inv in (False, True):
        assert np.array_equal(cr.ntt(x, inv), oracle.ntt(x, inv))


@pytest.mark.parametrize("kind", [False, "fork9", "zkevm"], ids=["config4", "fork9", "zkevm_shaped"])
def test_proof_with_cpuref_kernels_equals_oracle(oracle, cr, kind):
    """the whole proof with cpuref's LDE / NTT / Merkle / Steps-program kernels
    (cpuref.as_oracle_kernels) == the oracle's own proof; the Steps programs
    include the zkEVM-shaped ones (row shifts, shifted stores, F_p^3)"""
    import bench
    from oracle.stark_prover import OracleStark
    inst = bench.stark_instance(10, 1, 100, 16, kind)
    o = OracleStark(inst)
    o.witness()
    want = o.prove()
    with cr.as_oracle_kernels(oracle):
        f = OracleStark(inst)
        f.witness()
        got = f.prove()
    assert got == want
