"""GPU STARK (libzkgpu_stark over libzkgpu) vs the CPU oracle, bit-exact.

The whole proof -- roots, evals, FRI layers, every query opening, finalPol --
must be identical to the oracle's (which is itself verified as a valid proof
in test_stark_oracle.py), plus stage-level parity for the new kernels.
"""
import numpy as np
import pytest

from golden_replay import verify_fri

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001


def rand_gl(rng, shape):
    return rng.integers(0, 2**63, size=shape, dtype=np.uint64)


def oracle_proof(inst):
    from oracle.stark_prover import OracleStark
    o = OracleStark(inst)
    o.witness()
    return o, o.prove()


@pytest.mark.parametrize("n_bits,blow,t,m,q,q_deg", [(8, 1, 4, 2, 8, 2), (10, 1, 6, 3, 16, 2), (9, 2, 3, 1, 12, 2),
                                                     (12, 1, 10, 4, 32, 2), (13, 1, 4, 2, 24, 2),
                                                     (10, 2, 4, 2, 16, 4), (9, 3, 3, 1, 12, 7)])
def test_full_proof_bit_exact(oracle, zkgpu, n_bits, blow, t, m, q, q_deg):
    """q_deg > 2 (blowup 2^2 / 2^3): qq2 holds 3*q_deg columns (starks.cpp:233)."""
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import GpuStark
    inst = SyntheticStark(n_bits=n_bits, blowup_bits=blow, t=t, m=m, n_queries=q, q_deg=q_deg)
    o, ref = oracle_proof(inst)
    g = GpuStark(inst)
    assert np.array_equal(g.verkey(), o.verkey)
    assert np.array_equal(g.publics(), o.publics)
    g.witness()
    got = g.prove()
    for k in ref:
        assert got[k] == ref[k], k
    bad, _, _ = verify_fri(oracle, got, g.verkey(), g.publics(), inst.fri_steps, inst.n_queries)
    assert bad["s0"] == bad["fri_tree"] == bad["fold"] == bad["final"] == 0
    timers = g.timers()
    assert "STARK_STEP_1_LDE" in timers and timers["STARK_TOTAL"] > 0
    g.close()


def test_config4_shape_bit_exact(oracle, zkgpu):
    """The benchmarked config-4 instance shape (bench.stark_instance: 100 cm1
    columns, 2 plookups, post-Z step3, 128 queries, FRI steps nBitsExt, -4, ...)
    at 2^16 rows: GPU proof == oracle proof, and it verifies."""
    from bench import stark_instance
    from zkgpu.stark import GpuStark
    inst = stark_instance(16, 1, 100, 128)
    assert len(inst.fri_steps) >= 3 and inst.n_cm1 == 100 and inst.n_queries == 128
    o, ref = oracle_proof(inst)
    g = GpuStark(inst)
    g.witness()
    got = g.prove()
    for k in ref:
        assert got[k] == ref[k], k
    bad, _, _ = verify_fri(oracle, got, g.verkey(), g.publics(), inst.fri_steps, inst.n_queries)
    assert bad["s0"] == bad["fri_tree"] == bad["fold"] == bad["final"] == 0
    g.close()


def test_recursive1_shaped_proof_bit_exact(oracle, zkgpu):
    """The golden recursive1 proofs' structure at a small size: blowup 2^3,
    43 queries, FRI step reductions of 4 and 3 bits (golden: nBitsExt 20,
    steps [20, 16, 12, 9, 6]) -- here nBitsExt 14, steps [14, 10, 7, 4]."""
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import GpuStark
    inst = SyntheticStark(n_bits=11, blowup_bits=3, t=5, m=2, n_queries=43, fri_steps=[14, 10, 7, 4])
    o, ref = oracle_proof(inst)
    g = GpuStark(inst)
    g.witness()
    got = g.prove()
    for k in ref:
        assert got[k] == ref[k], k
    bad, _, _ = verify_fri(oracle, got, g.verkey(), g.publics(), inst.fri_steps, inst.n_queries)
    assert bad["s0"] == bad["fri_tree"] == bad["fold"] == bad["final"] == 0
    g.close()


def test_set_cm1_row_major_boundary(oracle, zkgpu):
    """Loading the trace through the reference's row-major layout gives the same proof."""
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import GpuStark
    inst = SyntheticStark(n_bits=9, t=3, m=1, n_queries=8)
    o, ref = oracle_proof(inst)
    g = GpuStark(inst)
    g.set_cm1(o.S[0])
    assert g.prove() == ref
    g.close()


def test_set_cm1_async_pipelined_proofs(oracle, zkgpu):
    """Back-to-back proofs with the next trace handed over in the background
    (zkgpu_stark_set_cm1_async during the current prove): each proof equals the
    oracle's proof of its own trace.  The two traces differ in the free
    (unconstrained) columns."""
    from oracle.stark_prover import OracleStark
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import GpuStark
    inst = SyntheticStark(n_bits=10, t=3, m=1, n_free=5, n_queries=8)
    free = list(range(3 * inst.t, 3 * inst.t + inst.n_free))
    traces, refs = [], []
    for k in range(3):
        o = OracleStark(inst)
        o.witness()
        if k:
            rng = np.random.default_rng(k)
            o.S[0][:, free] = rand_gl(rng, (o.N, len(free)))
        traces.append(o.S[0].copy())
        refs.append(o.prove())
    assert refs[0] != refs[1]
    g = GpuStark(inst)
    g.set_cm1(traces[0])
    assert np.array_equal(g.get_cm1(), traces[0])
    g.set_cm1_async(traces[1])  # loads while proof 0 runs, taken when it returns
    assert g.prove() == refs[0]
    assert np.array_equal(g.get_cm1(), traces[1])
    g.set_cm1_async(traces[2])
    assert g.prove() == refs[1]
    assert g.prove() == refs[2]
    assert g.prove() == refs[2]  # nothing queued: the trace stays
    # a queued load superseded by a synchronous one
    g.set_cm1_async(traces[1])
    g.set_cm1(traces[0])
    assert g.prove() == refs[0]
    # a queued load superseded by another queued one
    g.set_cm1_async(traces[1])
    g.set_cm1_async(traces[2])
    assert g.prove() == refs[0] and g.prove() == refs[2]
    # destroyed with a load still queued: the destructor waits for it
    g.set_cm1_async(traces[1])
    g.close()


def test_set_cm1_async_first_load_after_queued_work(oracle, zkgpu):
    """the first set_cm1_async allocates the second cm1 buffer and
    the loader stage, zeroed on the library stream.  With ~0.1 s of LDE work
    queued on that stream just before, those memsets run late; the loader's
    copies (its own non-blocking streams) must still land after them -- the
    queued trace is what the next proof sees."""
    import torch
    from oracle.stark_prover import OracleStark
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import GpuStark
    inst = SyntheticStark(n_bits=12, t=3, m=1, n_free=60, n_queries=8)
    free = list(range(3 * inst.t, 3 * inst.t + inst.n_free))
    o = OracleStark(inst)
    o.witness()
    trace = o.S[0].copy()
    trace[:, free] = rand_gl(np.random.default_rng(5), (o.N, len(free)))
    o.S[0][:] = trace
    want = o.prove()
    g = GpuStark(inst)
    g.witness()
    n, C = 1 << 22, 32
    src = torch.randint(0, 2**62, (C, n), dtype=torch.int64, device="cuda")
    out = torch.empty((C, 2 * n), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for _ in range(4):  # queued, not waited for
        zkgpu.extend_pol_dev(out, 2 * n, src, n, 2 * n, n, C)
    g.set_cm1_async(trace)
    g.prove()  # the witness's proof; the queued trace is taken when it returns
    assert np.array_equal(g.get_cm1(), trace)
    assert g.prove() == want
    g.close()
    del src, out


def test_lookup_value_not_in_table_fails_loudly(oracle, zkgpu):
    """An f value outside the table stops the GPU prover with the reference's
    "Number not included" error (polinomial.hpp:409-413)."""
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import GpuStark
    from zkgpu import ZkgpuError
    inst = SyntheticStark(n_bits=9, t=3, m=1, n_queries=8)
    o, _ = oracle_proof(inst)
    rows = o.S[0].copy()
    rows[9, inst.cm1_lk[2]] = 12345
    g = GpuStark(inst)
    g.set_cm1(rows)
    with pytest.raises(ZkgpuError, match="Number not included: w=9"):
        g.prove()
    g.close()


def test_calculate_z_dev(oracle, zkgpu):
    import torch
    rng = np.random.default_rng(3)
    n = 1 << 15
    num = rand_gl(rng, (n, 3))
    # den = num shifted by one row: the product closes
    den = np.roll(num, -1, axis=0)
    zref = np.zeros((n, 3), np.uint64)
    ok = oracle.lib().oc_calculate_z(oracle._p(zref), 3, oracle._p(num), 3, oracle._p(np.ascontiguousarray(den)), 3, n)
    assert ok
    dnum = zkgpu.to_device(np.ascontiguousarray(num.T))
    dden = zkgpu.to_device(np.ascontiguousarray(den.T))
    dz = torch.zeros((3, n), dtype=torch.int64, device="cuda:0")
    assert zkgpu.calculate_z_dev(dz, n, dnum, n, dden, n, n)
    assert np.array_equal(zkgpu.from_device(dz).T, zref)
    # a product that does not close is reported
    den2 = den.copy()
    den2[5, 0] ^= 3
    dden2 = zkgpu.to_device(np.ascontiguousarray(den2.T))
    assert not zkgpu.calculate_z_dev(dz, n, dnum, n, dden2, n, n)
    # the batched form (one read-back for a stage's grand products): the same
    # columns and verdicts, a failing product between closing ones
    dzs = [torch.zeros((3, n), dtype=torch.int64, device="cuda:0") for _ in range(3)]
    got = zkgpu.calculate_z_many_dev([(dzs[0], n, dnum, n, dden, n), (dzs[1], n, dnum, n, dden2, n),
                                      (dzs[2], n, dnum, n, dden, n)], n)
    assert got == [True, False, True]
    assert np.array_equal(zkgpu.from_device(dzs[0]).T, zref)
    assert np.array_equal(zkgpu.from_device(dzs[2]).T, zref)
    assert np.array_equal(zkgpu.from_device(dzs[1]), zkgpu.from_device(dz))
    assert zkgpu.calculate_z_many_dev([], n) == []
    assert zkgpu.calculate_z_many_dev([(dzs[0], n, dnum, n, dden2, n)], 0) == [True]  # an empty product


@pytest.mark.parametrize("world", [2, 4, 8])
def test_calculate_z_block_dev(oracle, zkgpu, world):
    """The row-sharded grand product (host/sharded_starks.hpp z_all): W
    blocks with z0 = 1, the scan of their totals, the blocks redone with
    z0 = prefix -> the whole-domain z, and the product of the totals closes."""
    import torch
    rng = np.random.default_rng(4 + world)
    n = (1 << 14) + 0
    num = rand_gl(rng, (n, 3))
    den = np.roll(num, -1, axis=0)
    zref = np.zeros((n, 3), np.uint64)
    assert oracle.lib().oc_calculate_z(oracle._p(zref), 3, oracle._p(num), 3, oracle._p(np.ascontiguousarray(den)),
                                       3, n)
    dnum = zkgpu.to_device(np.ascontiguousarray(num.T))
    dden = zkgpu.to_device(np.ascontiguousarray(den.T))
    dz = torch.zeros((3, n), dtype=torch.int64, device="cuda:0")
    nb = n // world
    tots = []
    for r in range(world):
        tots.append(zkgpu.calculate_z_block_dev(dz[:, r * nb:], n, dnum[:, r * nb:], n, dden[:, r * nb:], n, nb))
    pre = [1, 0, 0]
    for r in range(world):
        if r:
            zkgpu.calculate_z_block_dev(dz[:, r * nb:], n, dnum[:, r * nb:], n, dden[:, r * nb:], n, nb, pre)
        pre = [int(v) for v in oracle.gl3_mul(np.array(pre, np.uint64), tots[r])]
    assert pre == [1, 0, 0]
    assert np.array_equal(zkgpu.from_device(dz).T, zref)


def test_xdivxsub_dev(oracle, zkgpu):
    import torch
    rng = np.random.default_rng(4)
    nb, nbe = 11, 12
    ne = 1 << nbe
    xi = rand_gl(rng, 3)
    x = np.zeros(ne, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), 7, oracle.gl_w(nbe), ne)
    a = np.zeros((ne, 3), np.uint64)
    b = np.zeros((ne, 3), np.uint64)
    oracle.lib().oc_xdivxsub(oracle._p(a), oracle._p(b), oracle._p(x), ne, oracle._p(xi), oracle.gl_w(nb))
    da = torch.zeros(3 * ne, dtype=torch.int64, device="cuda:0")
    db = torch.zeros(3 * ne, dtype=torch.int64, device="cuda:0")
    zkgpu.xdivxsub_dev(da, db, xi, nb, nbe)
    torch.cuda.synchronize()
    assert np.array_equal(zkgpu.from_device(da).reshape(-1, 3), a)
    assert np.array_equal(zkgpu.from_device(db).reshape(-1, 3), b)


@pytest.mark.parametrize("n,eb", [(1 << 12, 1), (3 * 61440 + 777, 0)])
def test_evmap_dev(oracle, zkgpu, n, eb):
    """Several row blocks (61440 rows each) and a ragged tail; sub-entry
    groups of mixed size (dim-3 entries split into three)."""
    import ctypes
    rng = np.random.default_rng(6 + n)
    ne = n << eb
    cols = rand_gl(rng, (ne, 9))  # row-major for the oracle
    lev = rand_gl(rng, (n, 3))
    lpev = rand_gl(rng, (n, 3))
    entries = [(0, 1, 0), (1, 1, 1), (2, 3, 0), (2, 3, 1), (6, 1, 0), (5, 3, 1), (8, 1, 1), (7, 1, 0), (3, 3, 0)]
    ptrs = (ctypes.c_void_p * len(entries))(*[cols.ctypes.data + 8 * c for c, _, _ in entries])
    strides = np.full(len(entries), 9, np.uint64)
    dims = np.array([d for _, d, _ in entries], np.uint32)
    primes = np.array([p for _, _, p in entries], np.uint32)
    ref = np.zeros((len(entries), 3), np.uint64)
    oracle.lib().oc_evmap(oracle._p(ref), ctypes.cast(ptrs, ctypes.c_void_p), ctypes.c_void_p(strides.ctypes.data),
                          ctypes.c_void_p(dims.ctypes.data), ctypes.c_void_p(primes.ctypes.data), len(entries),
                          oracle._p(lev), oracle._p(lpev), n, eb)
    dcols = zkgpu.to_device(np.ascontiguousarray(cols.T))
    dlev = zkgpu.to_device(np.ascontiguousarray(lev.T))
    dlpev = zkgpu.to_device(np.ascontiguousarray(lpev.T))
    base = dcols.data_ptr()
    got = zkgpu.evmap_dev([base + 8 * ne * c for c, _, _ in entries], [ne] * len(entries), dims, primes, dlev, dlpev,
                          n, n, eb)
    assert np.array_equal(got, ref)


def _upload_sections(zkgpu, o):
    """Oracle sections (row-major) -> device column-major {index: (tensor, ld, ncols)}."""
    secs = {}
    for k, a in o.S.items():
        secs[k] = (zkgpu.to_device(np.ascontiguousarray(a.T)), a.shape[0], a.shape[1])
    return secs


@pytest.mark.parametrize("n_bits,blow", [(8, 1), (9, 2)])
def test_step42ns_stage(oracle, zkgpu, n_bits, blow):
    """Stage 4 piece by piece: constraint quotient on the 2^nBitsExt domain,
    INTT, quotient split, NTT (starks.cpp:226-296) vs the oracle's sections."""
    import torch
    from zkgpu.synthetic import SyntheticStark, SEC_Q_2NS
    inst = SyntheticStark(n_bits=n_bits, blowup_bits=blow, t=4, m=2, n_queries=8)
    o, _ = oracle_proof(inst)
    N, NE, eb = o.N, o.NE, o.eb
    secs = _upload_sections(zkgpu, o)
    q = torch.zeros((3, NE), dtype=torch.int64, device="cuda:0")
    secs[SEC_Q_2NS] = (q, NE, 3)
    zkgpu.zxp_eval_dev(inst.programs["step42ns"], secs, inst.n_bits_ext, o.challenges, o.publics,
                       extend_bits=eb, x_start=7)
    torch.cuda.synchronize()
    assert np.array_equal(zkgpu.from_device(q).T, o.S[10])
    qq1 = torch.zeros((3, NE), dtype=torch.int64, device="cuda:0")
    zkgpu.ntt_dev(qq1, NE, q, NE, NE, 3, inverse=True)
    ref_qq1 = oracle.ntt(o.S[10], True)
    assert np.array_equal(zkgpu.from_device(qq1).T, ref_qq1)
    qq2 = torch.zeros((inst.q_deg * 3, NE), dtype=torch.int64, device="cuda:0")
    shift_in = pow(pow(7, P - 2, P), N, P)
    zkgpu.qsplit_dev(qq2, NE, qq1, NE, N, inst.q_deg, shift_in)
    cm4 = torch.zeros((inst.q_deg * 3, NE), dtype=torch.int64, device="cuda:0")
    zkgpu.ntt_dev(cm4, NE, qq2, NE, NE, inst.q_deg * 3)
    torch.cuda.synchronize()
    assert np.array_equal(zkgpu.from_device(cm4).T, o.S[8])


@pytest.mark.parametrize("name", ["step1", "step2", "step3prev", "step42ns", "step52ns"])
@pytest.mark.parametrize("mode", [("1", "0", "2"), ("1", "0", "0"), ("1", "3", "0"), ("0", "0", "0")])
def test_zxp_programs_vs_oracle(oracle, zkgpu, name, mode, monkeypatch):
    """Each synthetic program on random sections: the GPU -- the run-time
    compiled straight-line kernel, the interpreter on the compiled program at
    the default / a tiny term cap, and the interpreter on the unfused source
    program -- equals the oracle's evaluation of the SOURCE program, bit for
    bit."""
    import ctypes
    import torch
    from zkgpu.synthetic import SyntheticStark
    monkeypatch.setenv("ZKGPU_ZXP_FUSE", mode[0])
    monkeypatch.setenv("ZKGPU_ZXP_MAX_TERMS", mode[1])
    monkeypatch.setenv("ZKGPU_ZXP_JIT", mode[2])
    inst = SyntheticStark(n_bits=9, blowup_bits=1, t=8, m=3, n_free=4, n_lookups=2, n_queries=8)
    prog = inst.programs[name]
    eb = inst.blowup_bits
    logd = inst.n_bits_ext if prog.domain_ext else inst.n_bits
    dom = 1 << logd
    rng = np.random.default_rng(sum(map(ord, name)))
    widths = {0: inst.n_cm1, 1: inst.n_cm2, 2: inst.n_cm3, 3: inst.n_tmp, 4: inst.n_const, 5: inst.n_cm1,
              6: inst.n_cm2, 7: inst.n_cm3, 8: inst.n_cm4, 9: inst.n_const, 10: 3, 11: 3}
    S = {k: rand_gl(rng, (dom, w)) for k, w in widths.items()}
    chal = rand_gl(rng, (8, 3))
    pub = rand_gl(rng, inst.n_publics)
    evals = rand_gl(rng, (len(inst.evmap), 3))
    xdiv = rand_gl(rng, (dom, 3))
    xdivw = rand_gl(rng, (dom, 3))
    x_start = 7 if prog.domain_ext else 1
    x = np.zeros(dom, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), x_start, oracle.gl_w(logd), dom)
    n = dom >> eb if prog.domain_ext else dom
    wE = oracle.gl_w(eb)
    zh = np.array([pow((pow(7, n, P) * pow(wE, i, P) - 1) % P, P - 2, P) for i in range(1 << eb)], np.uint64)
    # device copies (column-major) before the oracle writes its outputs
    secs = {k: (zkgpu.to_device(np.ascontiguousarray(a.T)), dom, a.shape[1]) for k, a in S.items()}
    dx = zkgpu.to_device(xdiv)
    dxw = zkgpu.to_device(xdivw)
    ins, opn = prog.arrays()
    sp = (ctypes.c_void_p * 12)()
    strides = np.zeros(12, np.uint64)
    for k, a in S.items():
        sp[k] = a.ctypes.data
        strides[k] = a.shape[1]
    p = oracle._p
    oracle.lib().oc_zxp_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                             max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ctypes.cast(sp, ctypes.c_void_p),
                             ctypes.c_void_p(strides.ctypes.data), dom, p(chal), p(pub), p(evals), p(x), p(xdiv),
                             p(xdivw), p(zh), zh.size)
    zkgpu.zxp_eval_dev(prog, secs, logd, chal, pub, evals, dx if prog.domain_ext else None,
                       dxw if prog.domain_ext else None, extend_bits=eb, x_start=x_start)
    torch.cuda.synchronize()
    for k, (t, _, _) in secs.items():
        assert np.array_equal(zkgpu.from_device(t).T, S[k]), "section %d" % k


def test_full_proof_bit_exact_jit(oracle, zkgpu, monkeypatch):
    """The whole proof with every expression program as a run-time compiled
    straight-line kernel (csrc/zxp_jit.hip) equals the oracle's proof."""
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import GpuStark
    monkeypatch.setenv("ZKGPU_ZXP_JIT", "2")
    inst = SyntheticStark(n_bits=10, blowup_bits=1, t=6, m=3, n_queries=16)
    o, ref = oracle_proof(inst)
    g = GpuStark(inst)
    g.witness()
    got = g.prove()
    for k in ref:
        assert got[k] == ref[k], k
    g.close()


def test_fork9_widths_proof_bit_exact_jit(oracle, zkgpu, monkeypatch):
    """The fork-9-width instance (751/168/408/6 columns) with every program
    compiled: its step2 / step42ns / step52ns are block-split kernels (>= 1,000
    instructions) with the LDS column cache (csrc/zxp_jit.hip
    lds_column_cache), the code objects prebuilt by tools/jit_prebuild.py."""
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import GpuStark
    monkeypatch.setenv("ZKGPU_ZXP_JIT", "2")
    inst = SyntheticStark.fork9(n_bits=10, n_queries=8)
    o, ref = oracle_proof(inst)
    g = GpuStark(inst)
    g.witness()
    got = g.prove()
    for k in ref:
        assert got[k] == ref[k], k
    g.close()


@pytest.mark.parametrize("row0,nrows", [(0, 1 << 11), (512, 1024), (1536, 512), (3, 1000)])
def test_xdivxsub_rows_dev(oracle, zkgpu, row0, nrows):
    """A row block of xDivXSub (the sharded prover's rank block) equals those
    rows of the whole-domain oracle; rows outside the block stay untouched."""
    import torch
    rng = np.random.default_rng(5)
    nb, nbe = 10, 11
    ne = 1 << nbe
    xi = rand_gl(rng, 3)
    x = np.zeros(ne, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), 7, oracle.gl_w(nbe), ne)
    a = np.zeros((ne, 3), np.uint64)
    b = np.zeros((ne, 3), np.uint64)
    oracle.lib().oc_xdivxsub(oracle._p(a), oracle._p(b), oracle._p(x), ne, oracle._p(xi), oracle.gl_w(nb))
    da = torch.full((3 * ne,), 7, dtype=torch.int64, device="cuda:0")
    db = torch.full((3 * ne,), 7, dtype=torch.int64, device="cuda:0")
    zkgpu.xdivxsub_rows_dev(da, db, xi, nb, nbe, row0, nrows)
    torch.cuda.synchronize()
    ga, gb = zkgpu.from_device(da).reshape(-1, 3), zkgpu.from_device(db).reshape(-1, 3)
    assert np.array_equal(ga[row0:row0 + nrows], a[row0:row0 + nrows])
    assert np.array_equal(gb[row0:row0 + nrows], b[row0:row0 + nrows])
    assert (ga[:row0] == 7).all() and (ga[row0 + nrows:] == 7).all()


@pytest.mark.parametrize("row0,nrows", [(0, 1 << 12), (1024, 1024), (77, 3000)])
def test_lagrange_xi_rows_dev(oracle, zkgpu, row0, nrows):
    """LEv / LpEv in closed form == the reference's INTT of the powers of xi
    and w xi (starks.cpp:308-324), on any row block; a base-field xi is
    refused (the prover interpolates then)."""
    import torch
    rng = np.random.default_rng(6)
    nbits = 12
    n = 1 << nbits
    xi = rand_gl(rng, 3)
    w = oracle.gl_w(nbits)
    ref = []
    for base in (xi, np.array([oracle.gl_mul(int(xi[0]), w), oracle.gl_mul(int(xi[1]), w),
                               oracle.gl_mul(int(xi[2]), w)], np.uint64)):
        pw = np.zeros((n, 3), np.uint64)
        acc = np.array([1, 0, 0], np.uint64)
        for k in range(n):
            pw[k] = acc
            acc = oracle.gl3_mul(acc, base)
        ref.append(oracle.ntt(pw, inverse=True))
    lev = torch.zeros((3, nrows), dtype=torch.int64, device="cuda:0")
    lpev = torch.zeros((3, nrows), dtype=torch.int64, device="cuda:0")
    zkgpu.lagrange_xi_rows_dev(lev, lpev, nrows, xi, nbits, row0, nrows)
    torch.cuda.synchronize()
    assert np.array_equal(zkgpu.from_device(lev).T, ref[0][row0:row0 + nrows])
    assert np.array_equal(zkgpu.from_device(lpev).T, ref[1][row0:row0 + nrows])
    with pytest.raises(zkgpu.ZkgpuError, match="base field"):
        zkgpu.lagrange_xi_rows_dev(lev, lpev, nrows, np.array([5, 0, 0], np.uint64), nbits, row0, nrows)
