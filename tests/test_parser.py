"""The reference's zkEVM Steps bytecode through the product converter, on the CPU.

The five programs of ZkevmSteps (op*/args* in
src/starkpil/zkevm/chelpers/zkevm.chelpers.<step>.parser.hpp: step2prev 2,094
ops, step3prev 6,673, step3 13,117, step42ns 18,546, step52ns 3,001) are read
from /root/reference at test time (never stored in the repository) and
checked three ways on the same random sections of the fork-9 memory map
 at 2^10 rows:

  * oracle/parser.c -- the AVX2 case tables restated as a scalar interpreter
    over the reference's flat memory layout;
  * zkgpu_parser_convert (the product converter) -> the oracle's ZXP
    evaluator, on the source program and on the compiled program
    (zkgpu_zxp_compile: fusion, SSA slots, store forwarding);
  * for step2prev, step3prev and step52ns, also the reference's own
    straight-line generated code (step2prev_first in zkevm.chelpers.step2.cpp,
    step3prev_first, step52ns_first), translated by tools/chelpers_zxp.py --
    an independent statement of the same expressions that pins the opcode
    semantics both other paths use.

All must agree bit for bit on every section the program writes.  The ISA
table the converter is generated from (csrc/parser_isa.inc) must equal a
fresh extraction from the reference's case tables.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import parser_isa  # noqa: E402

P = 0xFFFFFFFF00000001
REF = parser_isa.REF
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference bytecode (/root/reference) not present")

# fork-9 memory map: ZXP section, mapOffsets, mapSectionsN
SEC_CM1_N, SEC_CM2_N, SEC_CM3_N, SEC_TMP_N, SEC_CONST_N, SEC_CM1_2NS, SEC_CM2_2NS, SEC_CM3_2NS, SEC_CM4_2NS, \
    SEC_CONST_2NS, SEC_Q_2NS, SEC_F_2NS = range(12)
ZKEVM_MAP = [(SEC_CM1_N, 0, 751), (SEC_CM2_N, 6299844608, 168), (SEC_CM3_N, 7709130752, 408),
             (SEC_TMP_N, 11182014464, 389), (SEC_CM1_2NS, 14445182976, 751), (SEC_CM2_2NS, 27044872192, 168),
             (SEC_CM3_2NS, 29863444480, 408), (SEC_CM4_2NS, 36708548608, 6)]
N_CONST = 234  # constant_pols.hpp:835
N_BITS, N_BITS_EXT = 23, 24
N_PUBLICS = 48
LOG_DOM = 10


def _rand(rng, shape):
    return rng.integers(0, P, size=shape, dtype=np.uint64)


@pytest.fixture(scope="module")
def bytecode():
    return {name: parser_isa.load_bytecode(name) for name in parser_isa.PARSERS}


@pytest.fixture(scope="module")
def zp():
    import zkgpu
    import zkgpu.parser as zp
    zkgpu.lib()
    return zp


def test_isa_table_matches_reference(tmp_path):
    isa = parser_isa.extract()
    fresh = tmp_path / "parser_isa.inc"
    parser_isa.emit_inc(isa, str(fresh))
    committed = os.path.join(ROOT, "zkevm-prover_amd", "csrc", "parser_isa.inc")
    assert open(committed).read() == fresh.read_text()
    # every opcode of every case table is covered, and the tables have the
    # shapes the survey decoded
    assert sorted(isa["step42ns"]) == list(range(93))
    assert sorted(isa["step52ns"]) == list(range(22))
    assert sorted(isa["step3"]) == list(range(121))
    assert len(isa["step42ns"][87]["ops"]) == 8 and isa["step42ns"][88]["nargs"] == 47


def test_bytecode_headers(bytecode):
    sizes = parser_isa.header_sizes()
    for name, (ops, args) in bytecode.items():
        assert ops.size == sizes[name]["NOPS"] and args.size == sizes[name]["NARGS"], name
    assert bytecode["step42ns"][0].size == 18546


def _data(rng, name, prog_ext):
    """random sections of the fork-9 map (dom rows each), constants, scalars"""
    dom = 1 << LOG_DOM
    S = {sec: _rand(rng, (dom, w)) for sec, _, w in ZKEVM_MAP}
    const = _rand(rng, (dom, N_CONST))
    S[SEC_CONST_N] = const
    S[SEC_CONST_2NS] = const
    S[SEC_Q_2NS] = np.zeros((dom, 3), np.uint64)
    S[SEC_F_2NS] = np.zeros((dom, 3), np.uint64)
    sc = {"challenges": _rand(rng, (8, 3)), "publics": _rand(rng, N_PUBLICS), "evals": _rand(rng, (2048, 3)),
          "x": _rand(rng, dom), "zhinv": _rand(rng, 2), "xdiv": _rand(rng, (dom, 3)), "xdivw": _rand(rng, (dom, 3))}
    return S, sc


def _copy(S):
    return {k: v.copy() for k, v in S.items()}


def _run_oracle_parser(oracle, pid, ops, args, S, sc, tmps):
    dom = 1 << LOG_DOM
    ext = pid >= 3
    secs = [(off, w, S[sec]) for sec, off, w in ZKEVM_MAP]
    rc = oracle.parser_eval(pid, ops, args, secs, S[SEC_CONST_2NS if ext else SEC_CONST_N], dom,
                            1 << (N_BITS_EXT if ext else N_BITS), tmps[0], tmps[1], sc["challenges"],
                            sc["publics"], sc["evals"], sc["x"], sc["zhinv"], sc["xdiv"], sc["xdivw"],
                            S[SEC_Q_2NS], S[SEC_F_2NS])
    assert rc == 0, "oracle parser status %d" % rc


def _run_zxp(oracle, prog, S, sc, compiled=None):
    dom = 1 << LOG_DOM
    secs = (ctypes.c_void_p * 12)()
    strides = np.zeros(12, np.uint64)
    for k, a in S.items():
        secs[k] = a.ctypes.data
        strides[k] = a.shape[1]
    p = oracle._p
    L = oracle.lib()
    if compiled is None:
        ins, opn = prog.arrays()
        ins = np.ascontiguousarray(ins, np.uint32)
        opn = np.ascontiguousarray(opn, np.uint32)
        L.oc_zxp_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                      max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ctypes.cast(secs, ctypes.c_void_p),
                      ctypes.c_void_p(strides.ctypes.data), dom, p(sc["challenges"]), p(sc["publics"]),
                      p(sc["evals"]), p(sc["x"]), p(sc["xdiv"]), p(sc["xdivw"]), p(sc["zhinv"]), sc["zhinv"].size)
    else:
        c = compiled
        ins, opn = np.ascontiguousarray(c["instr"]), np.ascontiguousarray(c["opnd"])
        term = np.ascontiguousarray(c["term"])
        cst = np.ascontiguousarray(c["cst"]).reshape(-1)
        if cst.size == 0:
            cst = np.zeros(3, np.uint64)
        L.oc_zxc_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                      c["n_tmp1"], c["n_tmp3"], ctypes.c_void_p(term.ctypes.data if term.size else 0),
                      ctypes.c_void_p(cst.ctypes.data), ctypes.cast(secs, ctypes.c_void_p),
                      ctypes.c_void_p(strides.ctypes.data), dom, p(sc["challenges"]), p(sc["publics"]),
                      p(sc["evals"]), p(sc["x"]), p(sc["xdiv"]), p(sc["xdivw"]), p(sc["zhinv"]), sc["zhinv"].size)


def _written(prog):
    out = set()
    for op, d, a, b in prog.instr:
        kind, sec = prog.opnd[d][0], prog.opnd[d][1]
        if kind in (2, 3):  # ZXP_COL / ZXP_COL3
            out.add(sec)
    return out


@pytest.mark.parametrize("name", parser_isa.PARSERS)
def test_converter_equals_oracle_parser(oracle, zp, bytecode, name):
    import zkgpu
    pid = parser_isa.PARSERS.index(name)
    ops, args = bytecode[name]
    prog = zp.convert(pid, ops, args, ZKEVM_MAP, N_BITS, N_BITS_EXT)
    assert prog.domain_ext == (1 if pid >= 3 else 0)
    written = _written(prog)
    assert written, name
    rng = np.random.default_rng(0xB17E + pid)
    S0, sc = _data(rng, name, pid >= 3)
    A = _copy(S0)
    _run_oracle_parser(oracle, pid, ops, args, A, sc, (prog.n_tmp1, prog.n_tmp3))
    B = _copy(S0)
    _run_zxp(oracle, prog, B, sc)
    comp = zkgpu.zxp_compile(prog, sc["challenges"], sc["publics"], sc["evals"])
    C = _copy(S0)
    _run_zxp(oracle, prog, C, sc, compiled=comp)
    changed = 0
    for k in S0:
        assert np.array_equal(A[k], B[k]), "%s: section %d, converted program != oracle parser" % (name, k)
        assert np.array_equal(A[k], C[k]), "%s: section %d, compiled program != oracle parser" % (name, k)
        changed += int(not np.array_equal(A[k], S0[k]))
    assert changed == len(written), (name, written)


STRAIGHT = {"step2prev": ("zkevm.chelpers.step2.cpp", "step2prev_first"),
            "step3prev": ("zkevm.chelpers.step3prev.cpp", "step3prev_first"),
            "step52ns": ("zkevm.chelpers.step52ns.cpp", "step52ns_first")}


@pytest.mark.parametrize("name", sorted(STRAIGHT))
def test_bytecode_equals_reference_straight_line_code(oracle, bytecode, name):
    """The reference's generated per-row code for the same program (read as
    text, translated by tools/chelpers_zxp.py) gives the same sections as the
    oracle's bytecode interpreter: pins the case-table semantics."""
    from chelpers_zxp import translate_file
    pid = parser_isa.PARSERS.index(name)
    ext = pid >= 3
    fname, func = STRAIGHT[name]
    sections = {w: (sec, off) for sec, off, w in ZKEVM_MAP if (sec >= SEC_CM1_2NS) == ext}
    prog, _ = translate_file(os.path.join(REF, fname), func, sections, 1 if ext else 0)
    ops, args = bytecode[name]
    rng = np.random.default_rng(0x57A1 + pid)
    S0, sc = _data(rng, name, ext)
    A = _copy(S0)
    sizes = parser_isa.header_sizes()[name]
    _run_oracle_parser(oracle, pid, ops, args, A, sc, (sizes.get("NTEMP1", 4), sizes.get("NTEMP3", 4)))
    B = _copy(S0)
    _run_zxp(oracle, prog, B, sc)
    for k in S0:
        assert np.array_equal(A[k], B[k]), "%s: section %d, bytecode != straight-line code" % (name, k)


def test_synthetic_step42ns_converter_equals_oracle_parser(oracle, zp):
    """The step42ns-shaped program of zkgpu/synthetic_bytecode.py (the GPU
    tests' and the step42ns bench's program) through the converter == the
    oracle's case-table interpreter, on a 2^5-row domain.  The interpreters keep
    temporaries across rows (as the reference's do), so this also checks that
    the generator never reads a temporary before writing it in the row."""
    import zkgpu.synthetic_bytecode as sb
    shape = sb.load_shape()
    ops, args = sb.generate("step42ns", seed=1)
    secs = sb.sections(shape)
    prog = zp.convert(zp.STEP42NS, ops, args, secs, shape["n_bits"], shape["n_bits_ext"])
    dom = 1 << 5
    rng = np.random.default_rng(9)
    S = {sec: _rand(rng, (dom, w)) for sec, _, w in secs if sec >= 5}
    const = _rand(rng, (dom, shape["n_const"]))
    sc = {"challenges": _rand(rng, (8, 3)), "publics": _rand(rng, 48), "evals": _rand(rng, (4, 3)),
          "x": _rand(rng, dom), "zhinv": _rand(rng, 2), "xdiv": np.zeros((dom, 3), np.uint64),
          "xdivw": np.zeros((dom, 3), np.uint64)}
    qref = np.zeros((dom, 3), np.uint64)
    off = {sec: o for sec, o, _ in secs}
    rc = oracle.parser_eval(3, ops, args, [(off[s], a.shape[1], a) for s, a in S.items()], const, dom,
                            1 << shape["n_bits_ext"], shape["programs"]["step42ns"]["ntemp1"],
                            shape["programs"]["step42ns"]["ntemp3"], sc["challenges"], sc["publics"], sc["evals"],
                            sc["x"], sc["zhinv"], q=qref)
    assert rc == 0 and qref.any()
    B = {k: v.copy() for k, v in S.items()}
    B[SEC_CONST_2NS] = const
    B[SEC_Q_2NS] = np.zeros((dom, 3), np.uint64)
    global LOG_DOM
    saved, LOG_DOM = LOG_DOM, 5
    try:
        _run_zxp(oracle, prog, B, sc)
    finally:
        LOG_DOM = saved
    assert np.array_equal(B[SEC_Q_2NS], qref)


@pytest.mark.parametrize("name", ["step2prev", "step3prev", "step3", "step42ns", "step52ns"])
def test_synthetic_programs_converter_equals_oracle_parser(oracle, zp, name):
    """Every synthetic program of zkgpu/synthetic_bytecode.py (the shapes of
    the reference's five fork-9 programs: stage-2/3 column programs with
    shifted stores, the quotient, the FRI polynomial) through the converter
    and the ZXP compiler == the oracle's case-table interpreter on the fork-9
    map at 2^10 rows; and the compiled program is one the run-time compiled
    kernels take (no interpreter fallback on the GPU)."""
    import zkgpu
    import zkgpu.synthetic_bytecode as sb
    pid = parser_isa.PARSERS.index(name)
    ops, args = sb.generate(name, seed=1)
    prog = zp.convert(pid, ops, args, ZKEVM_MAP, N_BITS, N_BITS_EXT)
    written = _written(prog)
    assert written, name
    rng = np.random.default_rng(0x5E + pid)
    S0, sc = _data(rng, name, pid >= 3)
    A = _copy(S0)
    sh = sb.load_shape()["programs"][name]
    _run_oracle_parser(oracle, pid, ops, args, A, sc, (max(sh["ntemp1"], 8), max(sh["ntemp3"], 4)))
    B = _copy(S0)
    _run_zxp(oracle, prog, B, sc)
    comp = zkgpu.zxp_compile(prog, sc["challenges"], sc["publics"], sc["evals"])
    C = _copy(S0)
    _run_zxp(oracle, prog, C, sc, compiled=comp)
    changed = 0
    for k in S0:
        assert np.array_equal(A[k], B[k]), "%s: section %d, converted program != oracle parser" % (name, k)
        assert np.array_equal(A[k], C[k]), "%s: section %d, compiled program != oracle parser" % (name, k)
        changed += int(not np.array_equal(A[k], S0[k]))
    assert changed == len(written), (name, written)
    assert zkgpu.zxp_jit_source(prog, sc["challenges"], sc["publics"], sc["evals"])
