"""Pin the ZXP expression semantics against the reference's OWN generated step
code and golden proof (recursive1.zkin.proof_0.json).

The recursive1 circuit's per-row step code
(src/starkpil/starkRecursive1/chelpers/recursive1.chelpers.step{42,52}ns.cpp)
is translated at test time into ZXP programs (tools/chelpers_zxp.py; nothing
derived from it is stored in the repository), then:

  * step52ns, evaluated by the oracle's C ZXP evaluator at the 43 query rows
    from the rows the proof opens (s0_vals1/3/4/C, evals, xDivXSub at the query
    points), reproduces the FRI polynomial values in s1_vals -- the first FRI
    layer the reference committed (friProve.cpp:20-60);
  * step42ns, evaluated at xi over F_p^3 from the proof's evals (the verifier's
    view), satisfies the quotient identity q(xi) = sum_p xi^(pN) q_p(xi)
    (starks.cpp:226-296).
The GPU interpreter is bit-exact with the oracle evaluator on every synthetic
program (test_gpu_stark.py), so together these pin the GPU's semantics too.

CPU only; skipped when /root/reference is not present (it never is on the GPU
box, where nothing may read it).
"""
import ctypes
import os
import sys

import numpy as np
import pytest

from golden_replay import arr, load_meta, load_proof, transcript_challenges

REF = "/root/reference/src/starkpil/starkRecursive1/chelpers"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources not present")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

P = 0xFFFFFFFF00000001
N_BITS, N_BITS_EXT = 17, 20  # recursive1 starkStruct (golden_meta nBitsExt 20, blowup 8)


def _sections():
    from zkgpu.synthetic import SEC_CM1_2NS, SEC_CM3_2NS, SEC_CM4_2NS
    # row stride -> (section, base offset of the section in the reference's map);
    # widths match s0_vals1 (18), s0_vals3 (39), s0_vals4 (21)
    return {18: (SEC_CM1_2NS, 11010048), 39: (SEC_CM3_2NS, 29884416), 21: (SEC_CM4_2NS, 70778880)}


@pytest.fixture(scope="module")
def golden():
    meta = load_meta()
    name = "recursive1.zkin.proof_0.json"
    proof = load_proof(name)
    verkey = meta[meta["proofs"][name]["verkey"]]
    publics = list(proof["publics"]) + list(meta["recursive2_constRoot"])
    return meta, proof, verkey, publics


@pytest.fixture(scope="module")
def translated():
    import chelpers_zxp as cz
    secs = _sections()
    p52, _ = cz.translate_file(os.path.join(REF, "recursive1.chelpers.step52ns.cpp"), "step52ns_first", secs, 1)
    p42, _ = cz.translate_file(os.path.join(REF, "recursive1.chelpers.step42ns.cpp"), "step42ns_first", secs, 1)
    evmap = cz.evmap_from_step52ns(p52)
    return p52, p42, evmap


def test_evmap_recovered(golden, translated):
    _, proof, _, _ = golden
    _, _, evmap = translated
    assert sorted(evmap) == list(range(len(proof["evals"])))


def test_step52ns_reproduces_first_fri_layer(oracle, golden, translated):
    from zkgpu.synthetic import SEC_CM1_2NS, SEC_CM3_2NS, SEC_CM4_2NS, SEC_CONST_2NS, SEC_F_2NS
    meta, proof, verkey, publics = golden
    p52, _, _ = translated
    steps, nq = meta["friSteps"], meta["nQueries"]
    ch, _, ys = transcript_challenges(oracle, proof, verkey, publics, steps, nq)
    S = {SEC_CM1_2NS: arr(proof["s0_vals1"]).reshape(nq, -1), SEC_CM3_2NS: arr(proof["s0_vals3"]).reshape(nq, -1),
         SEC_CM4_2NS: arr(proof["s0_vals4"]).reshape(nq, -1), SEC_CONST_2NS: arr(proof["s0_valsC"]).reshape(nq, -1),
         SEC_F_2NS: np.zeros((nq, 3), np.uint64)}
    # x at the query rows: x_2ns[y] = 7 * w_NE^y (starks.hpp:147-183)
    wE = oracle.gl_w(N_BITS_EXT)
    x = np.array([7 * pow(wE, y, P) % P for y in ys], np.uint64)
    xi = np.ascontiguousarray(ch[7], np.uint64)
    xdiv = np.zeros((nq, 3), np.uint64)
    xdivw = np.zeros((nq, 3), np.uint64)
    L = oracle.lib()
    L.oc_xdivxsub(oracle._p(xdiv), oracle._p(xdivw), oracle._p(x), nq, oracle._p(xi), oracle.gl_w(N_BITS))
    chal = np.zeros((8, 3), np.uint64)
    for k, v in ch.items():
        chal[k] = v
    evals = arr(proof["evals"]).reshape(-1, 3)
    pub = np.array([int(v) for v in publics], np.uint64)
    ins, opn = p52.arrays()
    secs = (ctypes.c_void_p * 12)()
    strides = np.zeros(12, np.uint64)
    keep = {}
    for k, a in S.items():
        a = np.ascontiguousarray(a)
        keep[k] = a
        secs[k] = a.ctypes.data
        strides[k] = a.shape[1]
    zh = np.zeros(8, np.uint64)  # not used by step52ns
    L.oc_zxp_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                  max(p52.n_tmp1, 1), max(p52.n_tmp3, 1), ctypes.cast(secs, ctypes.c_void_p),
                  ctypes.c_void_p(strides.ctypes.data), nq, oracle._p(chal), oracle._p(pub), oracle._p(evals),
                  oracle._p(x), oracle._p(xdiv), oracle._p(xdivw), oracle._p(zh), 8)
    f = keep[SEC_F_2NS]
    s1 = arr(proof["s1_vals"]).reshape(nq, -1)
    for q, y in enumerate(ys):
        j = y >> steps[1]  # getTransposed: group y mod 2^steps[1], position y >> steps[1]
        assert [int(v) for v in f[q]] == [int(v) for v in s1[q, 3 * j:3 * j + 3]], q


# ---------------------------------------------------------------- F_p^3 at xi
def _m3(a, b):
    c = [0] * 5
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            c[i + j] += x * y
    c[2] += c[4]; c[1] += c[4]
    c[1] += c[3]; c[0] += c[3]
    return [v % P for v in c[:3]]


def _pow3(a, e):
    r = [1, 0, 0]
    while e:
        if e & 1:
            r = _m3(r, a)
        a = _m3(a, a)
        e >>= 1
    return r


def test_step42ns_quotient_identity_at_xi(oracle, golden, translated):
    from zkgpu.synthetic import ADD, SUB, MUL, COPY, TMP1, TMP3, COL, COL3, LIT, CHAL, PUB, X, ZI, SEC_Q_2NS
    meta, proof, verkey, publics = golden
    _, p42, evmap = translated
    steps, nq = meta["friSteps"], meta["nQueries"]
    ch, _, _ = transcript_challenges(oracle, proof, verkey, publics, steps, nq)
    ev = [[int(v) % P for v in e] for e in proof["evals"]]
    index = {(s, c, pr): k for k, (s, c, d, pr) in evmap.items()}
    xi = [int(v) for v in ch[7]]
    n = 1 << N_BITS
    zh = _pow3(xi, n)
    zh[0] = (zh[0] - 1) % P
    zinv = [int(v) for v in oracle.gl3_inv(np.array(zh, np.uint64))]
    opn = p42.opnd
    temps = {}
    out = None

    def val(i):
        kind, a, b, c = opn[i]
        if kind in (TMP1, TMP3):
            return temps[(kind, a)]
        if kind in (COL, COL3):
            return ev[index[(a, b, 1 if c else 0)]]
        if kind == LIT:
            return [(a | (b << 32)) % P, 0, 0]
        if kind == CHAL:
            return [int(v) for v in ch[a]]
        if kind == PUB:
            return [int(publics[a]) % P, 0, 0]
        if kind == X:
            return xi
        if kind == ZI:
            return zinv
        raise ValueError(kind)

    for op, dst, a, b in p42.instr:
        va = val(a)
        if op == COPY:
            r = va
        else:
            vb = val(b)
            if op == ADD:
                r = [(x + y) % P for x, y in zip(va, vb)]
            elif op == SUB:
                r = [(x - y) % P for x, y in zip(va, vb)]
            else:
                r = _m3(va, vb)
        kind, da = opn[dst][0], opn[dst][1]
        if kind in (TMP1, TMP3):
            temps[(kind, da)] = r
        else:
            assert kind == COL3 and da == SEC_Q_2NS
            out = r
    assert out is not None
    # q(xi) = sum_p xi^(pN) q_p(xi), q_p = cm4 pieces (starks.cpp:266-281)
    from zkgpu.synthetic import SEC_CM4_2NS
    q_deg = 7
    acc = [0, 0, 0]
    cur = [1, 0, 0]
    xin = _pow3(xi, n)
    for p in range(q_deg):
        acc = [(x + y) % P for x, y in zip(acc, _m3(cur, ev[index[(SEC_CM4_2NS, 3 * p, 0)]]))]
        cur = _m3(cur, xin)
    assert out == acc
