"""The ZXP compiler (zkgpu_zxp_compile, csrc/zxp_compile.cpp) against the
source programs, on the CPU.

zkgpu_zxp_eval_dev runs the COMPILED program on the GPU (linear-combination
fusion of Horner chains, SSA temporaries).  Here both the source program and
its compiled form are evaluated by the oracle's C evaluator (oracle/stark.c
oc_zxp_eval / oc_zxc_eval) on the same random sections, challenges, evals and
publics; every written section must be bit-identical.  Programs: all six of
the synthetic STARK (step0..step52ns) at several term caps, plus the
reference's own recursive1 step42ns / step52ns code translated at test time
when /root/reference is present (tests/test_chelpers_pin.py pins that code
against the golden proof).
"""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0xFFFFFFFF00000001


def _rand(rng, shape):
    return rng.integers(0, P, size=shape, dtype=np.uint64)


def _run(oracle, prog_arrays, compiled, widths, dom, rng_seed, consts):
    """Evaluate on fresh random sections; returns the sections after the run."""
    rng = np.random.default_rng(rng_seed)
    S = {k: _rand(rng, (dom, w)) for k, w in widths.items()}
    secs = (ctypes.c_void_p * 12)()
    strides = np.zeros(12, np.uint64)
    for k, a in S.items():
        secs[k] = a.ctypes.data
        strides[k] = a.shape[1]
    chal, pub, evals, x, xdiv, xdivw, zh = consts
    L = oracle.lib()
    p = oracle._p
    if compiled is None:
        ins, opn, nt1, nt3 = prog_arrays
        L.oc_zxp_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data), nt1, nt3,
                      ctypes.cast(secs, ctypes.c_void_p), ctypes.c_void_p(strides.ctypes.data), dom, p(chal), p(pub),
                      p(evals), p(x), p(xdiv), p(xdivw), p(zh), zh.size)
    else:
        c = compiled
        ins = np.ascontiguousarray(c["instr"])
        opn = np.ascontiguousarray(c["opnd"])
        term = np.ascontiguousarray(c["term"])
        cst = np.ascontiguousarray(c["cst"]).reshape(-1)
        if cst.size == 0:
            cst = np.zeros(3, np.uint64)
        L.oc_zxc_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                      c["n_tmp1"], c["n_tmp3"], ctypes.c_void_p(term.ctypes.data if term.size else 0),
                      ctypes.c_void_p(cst.ctypes.data), ctypes.cast(secs, ctypes.c_void_p),
                      ctypes.c_void_p(strides.ctypes.data), dom, p(chal), p(pub), p(evals), p(x), p(xdiv), p(xdivw),
                      p(zh), zh.size)
    return S


def _consts(rng, dom, n_pub, n_ev):
    return (_rand(rng, (8, 3)), _rand(rng, n_pub), _rand(rng, (max(n_ev, 1), 3)), _rand(rng, dom),
            _rand(rng, (dom, 3)), _rand(rng, (dom, 3)), _rand(rng, 2))


def _check_program(oracle, zkgpu_host, prog, widths, dom, n_pub, n_ev, max_terms, seed):
    rng = np.random.default_rng(seed)
    consts = _consts(rng, dom, n_pub, n_ev)
    chal, pub, evals = consts[0], consts[1], consts[2]
    comp = zkgpu_host.zxp_compile(prog, chal, pub, evals, max_terms=max_terms)
    ins, opn = prog.arrays()
    src = (np.ascontiguousarray(ins, np.uint32), np.ascontiguousarray(opn, np.uint32), max(prog.n_tmp1, 1),
           max(prog.n_tmp3, 1))
    want = _run(oracle, src, None, widths, dom, seed + 1, consts)
    got = _run(oracle, None, comp, widths, dom, seed + 1, consts)
    for k in widths:
        assert np.array_equal(want[k], got[k]), "section %d differs" % k
    return comp


@pytest.fixture(scope="module")
def zkgpu_host():
    import zkgpu
    zkgpu.lib()
    return zkgpu


def _synthetic_widths(inst):
    return {0: max(inst.n_cm1, 1), 1: max(inst.n_cm2, 1), 2: max(inst.n_cm3, 1), 3: max(inst.n_tmp, 1),
            4: inst.n_const, 5: max(inst.n_cm1, 1), 6: max(inst.n_cm2, 1), 7: max(inst.n_cm3, 1),
            8: inst.n_cm4, 9: inst.n_const, 10: 3, 11: 3}


@pytest.mark.parametrize("name", ["step0", "step1", "step2", "step3prev", "step42ns", "step52ns"])
@pytest.mark.parametrize("max_terms", [0, 3, 256])
def test_synthetic_programs(oracle, zkgpu_host, name, max_terms):
    from zkgpu.synthetic import SyntheticStark
    inst = SyntheticStark(n_bits=5, t=6, m=2, n_free=5, n_lookups=2, n_queries=4)
    prog = inst.programs[name]
    if not prog.instr:
        pytest.skip("empty program")
    dom = 1 << (inst.n_bits_ext if prog.domain_ext else inst.n_bits)
    _check_program(oracle, zkgpu_host, prog, _synthetic_widths(inst), dom, inst.n_publics, len(inst.evmap),
                   max_terms, seed=sum(map(ord, name)) + max_terms)


def test_fusion_shrinks_the_fri_program(zkgpu_host):
    """step52ns: the Horner chains become DOT instructions (far fewer ops)."""
    from zkgpu.synthetic import SyntheticStark
    inst = SyntheticStark(n_bits=5, t=30, m=2, n_free=8, n_lookups=2, n_queries=4)
    prog = inst.programs["step52ns"]
    comp = zkgpu_host.zxp_compile(prog, np.ones((8, 3), np.uint64) * 5, np.zeros(8, np.uint64),
                                  np.ones((len(inst.evmap), 3), np.uint64) * 3)
    ops = comp["instr"][:, 0]
    assert len(ops) * 10 < len(prog.instr)
    assert set(ops.tolist()) <= {2, 3, 4, 5}  # MUL (by xDivXSub), COPY, DOT1, DOT3


def test_compile_rejects_bad_programs(zkgpu_host):
    from zkgpu.synthetic import Program, COL, TMP1, ADD, LIT
    p = Program(0)
    p.op(ADD, p.lit(3), p.lit(4), p.lit(5))  # writes a literal
    with pytest.raises(RuntimeError):
        zkgpu_host.zxp_compile(p, np.zeros((8, 3), np.uint64), None)


def test_shifted_store_forwarding(oracle, zkgpu_host):
    """The reference's stage-3 parsers store a cell of the NEXT row
    (pols[off + ((i+1) % N) * stride], step3.parser.cpp opcodes 101-114) and
    read it back in the same row: the compiled program forwards the stored
    value and never re-reads a cell its row wrote.  As in the reference, the
    shifted value equals what row i+1 stores unshifted, so the parallel
    evaluation is deterministic; compiled == source on the oracle."""
    from zkgpu.synthetic import Program, ADD, SUB, MUL, COPY, SEC_CM1_N, SEC_TMP_N
    import zkgpu.synthetic as S
    p = Program(0)
    t = p.tmp1()
    u = p.tmp3()
    for sh in (1, 0):
        p.op(MUL, p.col(SEC_TMP_N, 0, sh), p.col(SEC_CM1_N, 1, sh), p.col(SEC_CM1_N, 2, sh))  # tmp0 = c1 c2
        p.op(MUL, u, p.col(SEC_TMP_N, 0, sh), p.chal(2))
        p.op(ADD, p.col3(SEC_TMP_N, 1, sh), u, p.col(SEC_CM1_N, 3, sh))  # tmp1..3 = tmp0 ch2 + c3
    p.op(ADD, t, p.col(SEC_TMP_N, 0, 1), p.col(SEC_TMP_N, 0))
    p.op(SUB, p.col(SEC_TMP_N, 4), t, p.col(SEC_TMP_N, 2, 1))
    p.op(MUL, p.col3(SEC_TMP_N, 5), p.col3(SEC_TMP_N, 1, 1), p.col3(SEC_TMP_N, 1))
    cp = _check_program(oracle, zkgpu_host, p, {0: 6, 3: 8}, 64, 1, 1, 0, seed=11)
    writes = {(o[1], o[2], o[3]) for (op, d, a, b) in cp["instr"] for o in [cp["opnd"][d]] if o[0] in (S.COL, S.COL3)}
    assert (SEC_TMP_N, 0, 1) in writes and (SEC_TMP_N, 1, 1) in writes
    srcs = []
    for (op, d, a, b) in cp["instr"]:
        if op in (4, 5):  # ZXP_DOT1 / ZXP_DOT3 (include/zkgpu_zxp.h)
            srcs += [int(tm["src"]) for tm in cp["term"][a:a + b] if int(tm["src"]) != 0xFFFFFFFF]
        else:
            srcs += [a] if op == COPY else [a, b]
    for x in srcs:
        o = cp["opnd"][x]
        if o[0] == S.COL:
            assert (o[1], o[2], o[3]) not in writes, o
        if o[0] == S.COL3:
            assert all((o[1], o[2] + c, o[3]) not in writes for c in range(3)), o


def test_column_write_hazard(oracle, zkgpu_host):
    """A pending form that reads column c must see the value from before a
    later store into c (read-before-write order of the source program)."""
    from zkgpu.synthetic import Program, ADD, SUB, MUL, COPY, SEC_CM1_N
    p = Program(0)
    t = p.tmp1()
    p.op(ADD, t, p.col(SEC_CM1_N, 0), p.col(SEC_CM1_N, 1))  # t = c0 + c1 (pending form)
    p.op(MUL, p.col(SEC_CM1_N, 0), p.col(SEC_CM1_N, 2), p.col(SEC_CM1_N, 3))  # c0 = c2 * c3
    u = p.tmp3()
    p.op(MUL, u, t, p.chal(1))  # uses the OLD c0
    p.op(ADD, u, u, p.col(SEC_CM1_N, 0))  # and the NEW c0
    p.op(COPY, p.col3(SEC_CM1_N, 4), u)
    p.op(SUB, p.col(SEC_CM1_N, 1), t, p.lit(1))
    _check_program(oracle, zkgpu_host, p, {0: 8}, 32, 1, 1, 0, seed=7)


# ---------------------------------------------------------------- reference step code
REF = "/root/reference/src/starkpil/starkRecursive1/chelpers"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources not present")
@pytest.mark.parametrize("which", ["step52ns", "step42ns"])
def test_reference_step_code(oracle, zkgpu_host, which):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import chelpers_zxp as cz
    from zkgpu.synthetic import SEC_CM1_2NS, SEC_CM3_2NS, SEC_CM4_2NS
    secs = {18: (SEC_CM1_2NS, 11010048), 39: (SEC_CM3_2NS, 29884416), 21: (SEC_CM4_2NS, 70778880)}
    prog, _ = cz.translate_file(os.path.join(REF, "recursive1.chelpers.%s.cpp" % which), "%s_first" % which, secs, 1)
    opn = np.array(prog.opnd, np.int64).reshape(-1, 4)
    widths = {}
    for kind, a, b, _c in opn:
        if kind in (2, 3):  # COL, COL3: section width from the highest column used
            widths[int(a)] = max(widths.get(int(a), 0), int(b) + (3 if kind == 3 else 1))
    n_ev = int(opn[opn[:, 0] == 8][:, 1].max()) + 1 if (opn[:, 0] == 8).any() else 1
    n_pub = int(opn[opn[:, 0] == 6][:, 1].max()) + 1 if (opn[:, 0] == 6).any() else 1
    comp = _check_program(oracle, zkgpu_host, prog, widths, 64, n_pub, n_ev, 0, seed=11)
    assert len(comp["instr"]) < len(prog.instr)


@pytest.mark.parametrize("name", ["step1", "step42ns", "step52ns"])
def test_jit_source_compiles_for_gfx950(zkgpu_host, name):
    """The straight-line kernel printed for a compiled program (csrc/zxp_jit.hip)
    compiles with hiprtc for gfx950 (no GPU needed); pointers and
    challenge-dependent values are not in the source."""
    from zkgpu.synthetic import SyntheticStark
    inst = SyntheticStark(n_bits=5, t=6, m=2, n_free=5, n_lookups=2, n_queries=4)
    prog = inst.programs[name]
    rng = np.random.default_rng(5)
    ch = _rand(rng, (8, 3))
    ev = _rand(rng, (len(inst.evmap), 3))
    src = zkgpu_host.zxp_jit_source(prog, ch, np.zeros(8, np.uint64), ev, rtc_check=True)
    assert "zxp_jit" in src
    src2 = zkgpu_host.zxp_jit_source(prog, _rand(rng, (8, 3)), np.zeros(8, np.uint64), _rand(rng, ev.shape))
    assert src == src2  # same structure -> same kernel (cached per process)


def test_fused_chains_only_for_fri_polynomials(zkgpu_host):
    """Fused column chains (csrc/zxp_jit.hip): the zkEVM-shaped FRI polynomial
    (three opening-point chains over 1,497 columns) prints its chains as loops
    reading each column once; the zkEVM-shaped quotient and the stage-3
    program (chains holding a small share of their column terms) are left
    alone; the kernel text does not depend on the challenges."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import jit_prebuild as jp
    ch, pub, ev = jp.consts()
    rng = np.random.default_rng(3)
    p52 = jp.program(1.0, "step52ns")
    src = zkgpu_host.zxp_jit_source(p52, ch, pub, ev)
    assert src.count("for (int q_") >= 3
    assert src == zkgpu_host.zxp_jit_source(p52, _rand(rng, ch.shape), pub, _rand(rng, ev.shape))
    for name in ("step3prev", "step42ns"):
        assert "for (int q_" not in zkgpu_host.zxp_jit_source(jp.program(0.25 if name == "step42ns" else 1.0, name),
                                                             ch, pub, ev)
