"""The lean HBM plan of the single-GPU prover (ZKGPU_MEM_LEAN,
include/zkgpu_stark.h; host/starks.cpp alloc_lean) and the in-place LDE it
rests on (zkgpu_gl_extend_pol_inplace_dev).

The plan shares one arena between the sections of stages 1-3 by their
lifetimes inside Starks::genProof (starks.cpp:49-224): cm1's stage-1 extension
is hashed and dropped, cm3 and (before stage 4) cm1 are extended in place over
their n-domain values, evmap reads the extended rows k << blowup with the
Lagrange weights of xi / 7 (starks.cpp:308-333).  Every proof must equal the
resident plan's and the oracle's bit for bit; the in-place LDE must equal the
out-of-place one with the column batches forced small (several batches, run
from the last down)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _inst(kind, bits=10, queries=16):
    import bench
    return bench.stark_instance(bits, 1, 100, queries, kind)


@pytest.mark.parametrize("logn,eb,ncols,batch", [(12, 1, 10, 3), (12, 2, 7, 2), (14, 1, 33, 0), (10, 3, 5, 1)])
def test_extend_pol_inplace_equals_out_of_place(zkgpu, logn, eb, ncols, batch):
    import torch
    n, ne = 1 << logn, 1 << (logn + eb)
    g = torch.Generator(device="cuda")
    g.manual_seed(logn * 100 + ncols)
    src = torch.randint(0, 2**63 - 1, (ncols, n), dtype=torch.int64, device="cuda", generator=g)
    ref = torch.empty((ncols, ne), dtype=torch.int64, device="cuda")
    base = torch.zeros(ncols * ne, dtype=torch.int64, device="cuda")
    base[:ncols * n].copy_(src.reshape(-1))
    zkgpu.set_lde_batch_cols(batch)
    try:
        zkgpu.extend_pol_dev(ref, ne, src, n, ne, n, ncols)
        zkgpu.extend_pol_inplace_dev(base, ne, n, ncols)
        torch.cuda.synchronize()
    finally:
        zkgpu.set_lde_batch_cols(0)
    assert torch.equal(base.reshape(ncols, ne), ref)


@pytest.fixture(scope="module")
def oracle_proofs(oracle):
    from oracle.stark_prover import OracleStark
    out = {}
    for kind in (False, "zkevm"):
        o = OracleStark(_inst(kind))
        o.witness()
        out[kind] = o.prove()
    return out


@pytest.mark.parametrize("kind", [False, "zkevm"], ids=["config4", "zkevm_shaped"])
@pytest.mark.parametrize("batch,keep", [(0, None), (7, "0"), (7, "45"), (0, "100000")],
                         ids=["batch_default-keep_auto", "batch7-keep0", "batch7-keep_part", "keep_all"])
def test_lean_proof_equals_oracle(zkgpu, oracle_proofs, monkeypatch, kind, batch, keep):
    """config-4 and the zkEVM-shaped instance at 2^10 under the lean plan
    (with the LDE batches forced to 7 columns: the in-place extensions of cm1
    (100 / 751 columns) and cm3 run in many batches; cm1's extended columns
    kept from stage 1: none -- all extended again at stage 4 --, some -- a
    two-region stage-1 tree --, all, or as many as the HBM holds) == the
    oracle's proof; and the trace is consumed: a second prove without a new
    trace fails, witness() then prove() gives the same proof again"""
    from zkgpu import ZkgpuError
    from zkgpu.stark import GpuStark, MEM_LEAN
    if keep is not None:
        monkeypatch.setenv("ZKGPU_LEAN_KEEP_COLS", keep)
    zkgpu.set_lde_batch_cols(batch)
    g = GpuStark(_inst(kind), mode=MEM_LEAN)
    try:
        assert g.memory_mode() == "lean"
        g.witness()
        p1 = g.prove()
        assert p1 == oracle_proofs[kind]
        with pytest.raises(ZkgpuError, match="consumed the trace"):
            g.prove_raw()
        with pytest.raises(ZkgpuError, match="consumed the trace"):
            g.get_cm1()
        g.witness()
        assert g.prove() == p1
    finally:
        zkgpu.set_lde_batch_cols(0)
        g.close()


def test_lean_set_cm1_and_refusals(zkgpu, oracle_proofs):
    """the executor hand-off under the lean plan: the resident prover's trace
    read back (get_cm1), loaded with set_cm1 into a lean prover, proves the
    same; set_cm1_async is refused loudly (its second cm1_n would not fit)"""
    from zkgpu import ZkgpuError
    from zkgpu.stark import GpuStark, MEM_LEAN, MEM_RESIDENT
    inst = _inst("zkevm")
    r = GpuStark(inst, mode=MEM_RESIDENT)
    try:
        assert r.memory_mode() == "resident"
        r.witness()
        rows = r.get_cm1()
        pr = r.prove()
        assert pr == r.prove()  # the resident plan keeps the trace
    finally:
        r.close()
    g = GpuStark(inst, mode=MEM_LEAN)
    try:
        with pytest.raises(ZkgpuError, match="not offered under the lean memory plan"):
            g.set_cm1_async(rows)
        for _ in range(2):
            g.set_cm1(rows)
            assert g.prove() == pr == oracle_proofs["zkevm"]
    finally:
        g.close()


def test_auto_plan_is_resident_when_it_fits(zkgpu):
    from zkgpu.stark import GpuStark
    g = GpuStark(_inst(False))
    try:
        assert g.memory_mode() == "resident"
    finally:
        g.close()


def test_lean_refused_when_the_quotient_reads_the_n_domain(zkgpu):
    """a stage-4 program that reads an n-domain section (other than the
    constants) cannot run under the lean plan: refused at create"""
    import copy
    from zkgpu import ZkgpuError
    from zkgpu.stark import GpuStark, MEM_LEAN
    from zkgpu import synthetic as sy
    inst = copy.deepcopy(_inst(False))
    p = inst.programs["step42ns"]
    a = p.o(sy.COL, sy.SEC_CM1_N, 0, 0)
    p.op(sy.ADD, p.o(sy.TMP1, 0, 0, 0), a, a)
    with pytest.raises(ZkgpuError, match="lean memory plan does not apply"):
        GpuStark(inst, mode=MEM_LEAN)


@pytest.mark.parametrize("ncols,split", [(100, 64), (751, 536), (13, 8), (9, 0)])
def test_merkletree_two_regions(zkgpu, ncols, split):
    """zkgpu_gl_merkletree2_dev (columns [0, split) in one region, the rest in
    another) == zkgpu_gl_merkletree_dev of the section in one piece"""
    import torch
    n = 1 << 10
    g = torch.Generator(device="cuda")
    g.manual_seed(ncols)
    src = torch.randint(0, 2**63 - 1, (ncols, n), dtype=torch.int64, device="cuda", generator=g)
    a = src[:split].contiguous() if split else torch.zeros((1, n), dtype=torch.int64, device="cuda")
    b = src[split:].contiguous()
    ref = torch.empty(zkgpu.merkle_num_elements(n), dtype=torch.int64, device="cuda")
    got = torch.empty_like(ref)
    zkgpu.merkletree_dev(ref, src, n, ncols, n)
    zkgpu.merkletree2_dev(got, a, b, n, split, ncols, n)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
