"""Steps bytecode on the GPU (include/zkgpu_parser.h) vs the oracle's
case-table interpreter (oracle/parser.c), bit for bit.

The reference's fork-9 programs cannot travel to the GPU box; the programs
here are built by zkgpu/synthetic_bytecode.py with the shape of the
reference's step42ns (its opcode histogram, temporaries, the fork-9 memory
map, next-row reads at shift 2 on the 2^24 domain: tests/golden/
zkevm_bytecode_shape.json) and go through the same product converter.  On the
CPU, tests/test_parser.py checks the converter on the reference's own five
programs.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001
SEC_CONST_2NS, SEC_Q_2NS = 9, 10


def _rand(rng, shape):
    return rng.integers(0, P, size=shape, dtype=np.uint64)


@pytest.mark.parametrize("log_dom,jit", [(12, "1"), (16, "0")])
def test_step42ns_shaped_program_gpu_equals_oracle(oracle, zkgpu, log_dom, jit, monkeypatch):
    """2^12: the LDS interpreter; 2^16 with ZKGPU_ZXP_JIT=0: the interpreter on
    a multi-workgroup domain (the compiled kernel is test_step42ns_shaped_jit)"""
    import torch
    monkeypatch.setenv("ZKGPU_ZXP_JIT", jit)
    import zkgpu.parser as zp
    import zkgpu.synthetic_bytecode as sb
    shape = sb.load_shape()
    ops, args = sb.generate("step42ns", seed=1)
    secs = sb.sections(shape)
    prog = zp.convert(zp.STEP42NS, ops, args, secs, shape["n_bits"], shape["n_bits_ext"])
    dom = 1 << log_dom
    rng = np.random.default_rng(log_dom)
    S = {sec: _rand(rng, (dom, w)) for sec, _, w in secs if sec >= 5}
    const = _rand(rng, (dom, shape["n_const"]))
    chal = _rand(rng, (8, 3))
    pub = _rand(rng, 48)
    evals = _rand(rng, (4, 3))
    # GPU: column-major device sections, the x / zhInv of a 2^log_dom coset domain
    dsecs = {sec: (zkgpu.to_device(np.ascontiguousarray(a.T)), dom, a.shape[1]) for sec, a in S.items()}
    dsecs[SEC_CONST_2NS] = (zkgpu.to_device(np.ascontiguousarray(const.T)), dom, const.shape[1])
    q = torch.zeros((3, dom), dtype=torch.int64, device="cuda:0")
    dsecs[SEC_Q_2NS] = (q, dom, 3)
    zkgpu.zxp_eval_dev(prog, dsecs, log_dom, chal, pub, evals, extend_bits=1, x_start=7)
    torch.cuda.synchronize()
    got = zkgpu.from_device(q).T
    # oracle: the same x_i = 7 w^i and zhInv of the 2^log_dom domain
    x = np.zeros(dom, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), 7, oracle.gl_w(log_dom), dom)
    n = dom >> 1
    zh = np.array([pow((pow(7, n, P) * pow(P - 1, i, P) - 1) % P, P - 2, P) for i in range(2)], np.uint64)
    qref = np.zeros((dom, 3), np.uint64)
    off = {sec: o for sec, o, _ in secs}
    sections = [(off[sec], a.shape[1], a) for sec, a in S.items()]
    rc = oracle.parser_eval(3, ops, args, sections, const, dom, 1 << shape["n_bits_ext"], 1196, 175, chal, pub,
                            evals, x, zh, q=qref)
    assert rc == 0
    assert qref.any()
    assert np.array_equal(got, qref)


def test_steps_parser_eval_host_dropin(oracle, zkgpu):
    """zkgpu_steps_parser_eval on the reference's host layout (one flat
    row-major memory map, StepsParams.pols, sections at mapOffsets) == the
    oracle parser on the same buffer, for a 2^13-row extended domain."""
    import copy
    import zkgpu.parser as zp
    import zkgpu.synthetic_bytecode as sb
    shape = copy.deepcopy(sb.load_shape())
    shape["n_bits"], shape["n_bits_ext"] = 12, 13
    dom = 1 << shape["n_bits_ext"]
    base = 0
    for m in shape["map"]:  # a compact map: the 2ns sections back to back, the rest unused
        if m["zxp_section"] >= 5:
            m["offset"] = base
            base += dom * m["width"]
        else:
            m["offset"] = 1 << 40
    ops, args = sb.generate("step42ns", seed=3, shape=shape)
    secs = sb.sections(shape)
    rng = np.random.default_rng(5)
    pols = _rand(rng, base)
    const = _rand(rng, (dom, shape["n_const"]))
    chal = _rand(rng, (8, 3))
    pub = _rand(rng, 48)
    q = np.zeros((dom, 3), np.uint64)
    zp.steps_eval(zp.STEP42NS, ops, args, secs, shape["n_bits"], shape["n_bits_ext"], pols, const, chal, pub,
                  q_2ns=q)
    x = np.zeros(dom, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), 7, oracle.gl_w(shape["n_bits_ext"]), dom)
    n = dom >> 1
    zh = np.array([pow((pow(7, n, P) * pow(P - 1, i, P) - 1) % P, P - 2, P) for i in range(2)], np.uint64)
    qref = np.zeros((dom, 3), np.uint64)
    sections = [(o, w, pols[o:o + dom * w].reshape(dom, w)) for sec, o, w in secs if sec >= 5]
    rc = oracle.parser_eval(3, ops, args, sections, const, dom, dom, 1196, 175, chal, pub, np.zeros((4, 3), np.uint64),
                            x, zh, q=qref)
    assert rc == 0 and qref.any()
    assert np.array_equal(q, qref)


@pytest.mark.parametrize("scale", [0.25, 1.0])
def test_step42ns_shaped_jit_gpu_equals_oracle(oracle, zkgpu, monkeypatch, scale):
    """the compiled expression kernels (csrc/zxp_jit.hip) of the step42ns-shaped
    program at 2^16 rows == the oracle parser: a quarter of step42ns's opcode
    counts (5.3 K ops, one kernel) and the full size (20 K ops, the kernel
    bench.py times at 2^24: segments, csrc/zxp_segment.cpp, their carried
    values through scratch columns).  The kernels come from the on-disk cache
    build() fills (tools/jit_prebuild.py; hiprtc takes minutes at this size),
    as the reference ships its expression code compiled."""
    import torch
    import zkgpu.parser as zp
    import zkgpu.synthetic_bytecode as sb
    monkeypatch.setenv("ZKGPU_ZXP_JIT", "2")
    shape = sb.load_shape()
    ops, args = sb.generate("step42ns", seed=1, scale=scale)
    secs = sb.sections(shape)
    prog = zp.convert(zp.STEP42NS, ops, args, secs, shape["n_bits"], shape["n_bits_ext"])
    rng = np.random.default_rng(0)
    assert zkgpu.zxp_jit_cached(prog, _rand(rng, (8, 3)), _rand(rng, 48), _rand(rng, (4, 3))), \
        "compiled kernel not cached: run build() (tools/jit_prebuild.py)"
    log_dom = 16
    dom = 1 << log_dom
    rng = np.random.default_rng(77)
    S = {sec: _rand(rng, (dom, w)) for sec, _, w in secs if sec >= 5}
    const = _rand(rng, (dom, shape["n_const"]))
    chal, pub, evals = _rand(rng, (8, 3)), _rand(rng, 48), _rand(rng, (4, 3))
    dsecs = {sec: (zkgpu.to_device(np.ascontiguousarray(a.T)), dom, a.shape[1]) for sec, a in S.items()}
    dsecs[SEC_CONST_2NS] = (zkgpu.to_device(np.ascontiguousarray(const.T)), dom, const.shape[1])
    q = torch.zeros((3, dom), dtype=torch.int64, device="cuda:0")
    dsecs[SEC_Q_2NS] = (q, dom, 3)
    zkgpu.prof_reset()
    zkgpu.prof_enable(True)
    zkgpu.zxp_eval_dev(prog, dsecs, log_dom, chal, pub, evals, extend_bits=1, x_start=7)
    torch.cuda.synchronize()
    zkgpu.prof_enable(False)
    ran = [k for k in zkgpu.prof_kernels() if k.startswith("k_zxp_jit")]
    if scale == 1.0:
        assert len(ran) > 1 and "k_zxp_jit_s00" in ran, ("the segmented kernels did not run", ran)
    else:
        assert ran == ["k_zxp_jit"], ("the compiled kernel did not run", ran)
    got = zkgpu.from_device(q).T
    x = np.zeros(dom, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), 7, oracle.gl_w(log_dom), dom)
    n = dom >> 1
    zh = np.array([pow((pow(7, n, P) * pow(P - 1, i, P) - 1) % P, P - 2, P) for i in range(2)], np.uint64)
    qref = np.zeros((dom, 3), np.uint64)
    off = {sec: o for sec, o, _ in secs}
    rc = oracle.parser_eval(3, ops, args, [(off[sec], a.shape[1], a) for sec, a in S.items()], const, dom,
                            1 << shape["n_bits_ext"], 1196, 175, chal, pub, evals, x, zh, q=qref)
    assert rc == 0 and qref.any()
    assert np.array_equal(got, qref)


# fork-9 map sections of the n-domain programs
STAGE = ["step2prev", "step3prev", "step3"]


@pytest.mark.parametrize("name", STAGE + ["step52ns"])
@pytest.mark.parametrize("log_dom,jit", [(12, "1"), (16, "2")])
def test_zkevm_shaped_programs_gpu_equal_oracle(oracle, zkgpu, monkeypatch, name, log_dom, jit):
    """The stage-2/3 column programs (step2prev / step3prev / step3: the
    reference's opcode mix, ~300 written cm3/tmpExp columns, shifted stores
    101-119 landing on row i+1 mod N) and the FRI polynomial (step52ns, 2,000
    evals, xDivXSub) of zkgpu/synthetic_bytecode.py on the GPU == the oracle's
    case-table interpreter, every section bit for bit: 2^12 rows through the
    interpreter, 2^16 through the run-time compiled kernels (segments for the
    large ones)."""
    import torch
    import zkgpu.parser as zp
    import zkgpu.synthetic_bytecode as sb
    monkeypatch.setenv("ZKGPU_ZXP_JIT", jit)
    shape = sb.load_shape()
    pid = sb.PARSERS.index(name)
    ext = pid >= 3
    ops, args = sb.generate(name, seed=1)
    secs = sb.sections(shape)
    prog = zp.convert(pid, ops, args, secs, shape["n_bits"], shape["n_bits_ext"])
    dom = 1 << log_dom
    rng = np.random.default_rng(1000 * pid + log_dom)
    S = {sec: _rand(rng, (dom, w)) for sec, _, w in secs if (sec >= 5) == ext}
    const = _rand(rng, (dom, shape["n_const"]))
    chal, pub, evals = _rand(rng, (8, 3)), _rand(rng, 48), _rand(rng, (2048, 3))
    xdiv, xdivw = (_rand(rng, (dom, 3)), _rand(rng, (dom, 3))) if ext else (None, None)
    csec = SEC_CONST_2NS if ext else 4
    dsecs = {sec: (zkgpu.to_device(np.ascontiguousarray(a.T)), dom, a.shape[1]) for sec, a in S.items()}
    dsecs[csec] = (zkgpu.to_device(np.ascontiguousarray(const.T)), dom, const.shape[1])
    f = torch.zeros((3, dom), dtype=torch.int64, device="cuda:0")
    if ext:
        dsecs[11] = (f, dom, 3)
    dx = zkgpu.to_device(xdiv) if ext else None
    dxw = zkgpu.to_device(xdivw) if ext else None
    zkgpu.prof_reset()
    zkgpu.prof_enable(True)
    zkgpu.zxp_eval_dev(prog, dsecs, log_dom, chal, pub, evals, xdiv=dx, xdivw=dxw, extend_bits=1 if ext else 0,
                       x_start=7 if ext else 1)
    torch.cuda.synchronize()
    zkgpu.prof_enable(False)
    ran = zkgpu.prof_kernels()
    if jit == "2":
        assert any(k.startswith("k_zxp_jit") for k in ran), ("the compiled kernels did not run", ran)
        if name == "step52ns":  # its three opening-point chains run fused (zxp_jit.hip "fused column chains")
            assert "for (int q_" in zkgpu.zxp_jit_source(prog, chal, pub, evals)
    # oracle on the same inputs (x_i = 7 w^i on the 2n coset, w^i on the n domain)
    x = np.zeros(dom, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), 7 if ext else 1, oracle.gl_w(log_dom), dom)
    zh = np.array([pow((pow(7, dom >> 1, P) * pow(P - 1, i, P) - 1) % P, P - 2, P) for i in range(2)], np.uint64)
    off = {sec: o for sec, o, _ in secs}
    R = {sec: a.copy() for sec, a in S.items()}
    fref = np.zeros((dom, 3), np.uint64)
    sh = shape["programs"][name]
    rc = oracle.parser_eval(pid, ops, args, [(off[sec], a.shape[1], a) for sec, a in R.items()], const, dom,
                            1 << (shape["n_bits_ext"] if ext else shape["n_bits"]), max(sh["ntemp1"], 8),
                            max(sh["ntemp3"], 4), chal, pub, evals, x, zh,
                            xdiv if ext else np.zeros((dom, 3), np.uint64),
                            xdivw if ext else np.zeros((dom, 3), np.uint64), f=fref)
    assert rc == 0
    if ext:
        assert fref.any()
        assert np.array_equal(zkgpu.from_device(f).T, fref)
    else:
        changed = 0
        for sec, a in R.items():
            got = zkgpu.from_device(dsecs[sec][0]).T
            assert np.array_equal(got, a), "%s: section %d differs" % (name, sec)
            changed += int(not np.array_equal(a, S[sec]))
        assert changed >= 1
