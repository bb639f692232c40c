"""Verifier-side replay of a whole STARK proof of a SyntheticStark /
zkEVM-shaped instance (test infrastructure: the CPU oracle is the checker).

What a verifier can re-derive from the proof, the instance's public
description (its step52ns program and evaluation map) and the verkey:
  * the Fiat-Shamir transcript of Starks::genProof (starks.cpp:28-29, 60,
    68-69, 141, 150-151, 222, 234, 293, 306, 336-342) and FRIProve::prove
    (friProve.cpp:30, 125, 130-133), then the query indices
    (getPermutations, friProve.cpp:156) -- tests/golden_replay.verify_fri;
  * every Merkle opening: the four stage trees and the constant tree at the
    query rows, every FRI layer tree (merkleTreeGL.cpp:12-35);
  * every FRI fold down to finalPol (friProve.cpp:44-108);
  * the FRI polynomial at every query row: step52ns (starks.cpp:371) run by
    the oracle's expression interpreter on the opened s0 values, the proof's
    evals, the transcript's challenges and xDivXSub at x = 7 w^y
    (starks.cpp:344-366), equal to the value FRI layer 1 opens at that row;
  * the degree of finalPol: f = sum of (p(x) - p(xi)) / (x - xi) terms over
    polynomials of degree < N has degree < N exactly when every eval is p(xi)
    (else the division leaves a pole, i.e. a high-degree remainder on the
    domain), so after the folds to 2^s elements only the 2^(s - blowup) lowest
    coefficients may be non-zero (the FRI low-degree claim, friProve.cpp:183).
    Only where step52ns IS that sum (the synthetic config-4 instance,
    zkgpu/synthetic.py): the zkEVM-shaped instance's step52ns is a program
    with the reference's opcode histogram, not its FRI polynomial
    (zkgpu/zkevm_shaped.py), so its f is not of low degree (low_degree=False).
  * the constraint identity at xi (starks.cpp:222-241; the verifier's check
    of the pil2/pilcom verifier circuits): step42ns run over F_p^3 at the
    single point xi with every column operand read from the proof's evals
    (row shift 0 -> the eval at xi, the next row -> at w xi, evMap's prime),
    Z_H^-1 -> (xi^N - 1)^-1, equals q(xi) = sum_p xi^(pN) q_p(xi) from the
    quotient pieces' evals.  Also only for the synthetic config-4 instance:
    it is a valid AIR (its trace satisfies its constraints); the zkEVM-shaped
    trace does not satisfy its stand-in constraints.
"""
import ctypes

import numpy as np

import golden_replay as gr

P = 0xFFFFFFFF00000001
SEC_TAGS = {5: "1", 6: "2", 7: "3", 8: "4", 9: "C"}  # s0 trees by 2ns section (include/zkgpu_zxp.h)


def _a2(x, width):
    return np.array([[int(v) for v in row] for row in x], dtype=np.uint64).reshape(-1, width)


def fri_pol_at_rows(oc, inst, proof, ys, ch, publics):
    """step52ns at the query rows from the proof's openings: (Q x 3)"""
    prog = inst.programs["step52ns"]
    ins, opn = prog.arrays()
    for kind, a, b, c in opn.tolist():
        if kind in (2, 3) and c != 0:
            raise AssertionError("step52ns reads column (%d, %d) at row shift %d: not a per-row program" % (a, b, c))
    Q = len(ys)
    widths = {5: inst.n_cm1, 6: inst.n_cm2, 7: inst.n_cm3, 8: inst.n_cm4, 9: inst.n_const}
    S = {k: np.zeros((Q, 1), np.uint64) for k in range(12)}
    for sec, tag in SEC_TAGS.items():
        S[sec] = np.ascontiguousarray(_a2(proof["s0_vals" + tag], widths[sec]))
    S[11] = np.zeros((Q, 3), np.uint64)
    secs = (ctypes.c_void_p * 12)()
    strides = np.zeros(12, np.uint64)
    for k, a in S.items():
        secs[k] = a.ctypes.data
        strides[k] = a.shape[1]
    L = oc.lib()
    wE = oc.gl_w(inst.n_bits_ext)
    x = np.array([7 * pow(wE, y, P) % P for y in ys], np.uint64)
    xi = np.ascontiguousarray(ch[7], dtype=np.uint64)
    xdiv = np.zeros((Q, 3), np.uint64)
    xdivw = np.zeros((Q, 3), np.uint64)
    L.oc_xdivxsub(oc._p(xdiv), oc._p(xdivw), oc._p(x), Q, oc._p(xi), oc.gl_w(inst.n_bits))
    chal = np.ascontiguousarray(np.array([ch[k] for k in range(8)], dtype=np.uint64))
    evals = np.ascontiguousarray(_a2(proof["evals"], 3))
    pub = np.ascontiguousarray(np.array([int(v) for v in publics] or [0], dtype=np.uint64))
    zh = np.ones(1, np.uint64)
    L.oc_zxp_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                  max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ctypes.cast(secs, ctypes.c_void_p),
                  ctypes.c_void_p(strides.ctypes.data), Q, oc._p(chal), oc._p(pub), oc._p(evals), oc._p(x),
                  oc._p(xdiv), oc._p(xdivw), oc._p(zh), 1)
    return S[11]


def final_degree_ok(oc, inst, proof):
    """finalPol (2^s evaluations on its coset) interpolates to degree < 2^(s - blowup)"""
    s = inst.fri_steps[-1]
    fp = _a2(proof["finalPol"], 3)
    coef = oc.ntt(np.ascontiguousarray(fp), True)
    lim = 1 << (s - (inst.n_bits_ext - inst.n_bits))
    return bool(np.all(coef[lim:] == 0)), int(np.count_nonzero(np.any(coef[lim:] != 0, axis=1)))


def _f3_mul(a, b):
    c0 = a[0] * b[0]
    c1 = a[0] * b[1] + a[1] * b[0]
    c2 = a[0] * b[2] + a[1] * b[1] + a[2] * b[0]
    c3 = a[1] * b[2] + a[2] * b[1]
    c4 = a[2] * b[2]
    return ((c0 + c3) % P, (c1 + c3 + c4) % P, (c2 + c4) % P)  # x^3 = x + 1


def _f3_pow(a, e):
    r = (1, 0, 0)
    while e:
        if e & 1:
            r = _f3_mul(r, a)
        a = _f3_mul(a, a)
        e >>= 1
    return r


def _f3_inv(a):
    return _f3_pow(a, P ** 3 - 2)


def quotient_identity(inst, proof, ch, publics):
    """(C(xi) Z_H(xi)^-1, q(xi)) from the proof's evals (module doc): step42ns
    interpreted over F_p^3 (ops and operands of include/zkgpu_zxp.h)"""
    from zkgpu import synthetic as sy
    evals = [tuple(int(v) % P for v in e) for e in proof["evals"]]
    chal = {k: tuple(int(v) for v in ch[k]) for k in ch}
    xi = chal[7]
    n = 1 << inst.n_bits
    xin = _f3_pow(xi, n)
    zi = _f3_inv(((xin[0] - 1) % P, xin[1], xin[2]))
    nxt = 1 << inst.blowup_bits
    prog = inst.programs["step42ns"]
    regs, out = {}, {}

    def val(i):
        kind, a, b, c = prog.opnd[i]
        if kind in (sy.TMP1, sy.TMP3):
            return regs[i]
        if kind in (sy.COL, sy.COL3):
            if c not in (0, nxt):
                raise AssertionError("step42ns reads column (%d, %d) at row shift %d" % (a, b, c))
            return evals[inst.ev_index[(a, b, 0 if c == 0 else 1)]]
        if kind == sy.LIT:
            return ((a | (b << 32)) % P, 0, 0)
        if kind == sy.CHAL:
            return chal[a]
        if kind == sy.PUB:
            return (int(publics[a]) % P, 0, 0)
        if kind == sy.X:
            return xi
        if kind == sy.EVAL:
            return evals[a]
        if kind == sy.ZI:
            return zi
        raise AssertionError("step42ns operand kind %d at xi" % kind)

    for op, dst, a, b in prog.instr:
        x = val(a)
        if op == sy.COPY:
            r = x
        else:
            y = val(b)
            if op == sy.ADD:
                r = tuple((u + v) % P for u, v in zip(x, y))
            elif op == sy.SUB:
                r = tuple((u - v) % P for u, v in zip(x, y))
            else:
                r = _f3_mul(x, y)
        if prog.opnd[dst][0] in (sy.TMP1, sy.TMP3):
            regs[dst] = r
        else:
            out[prog.opnd[dst][1:]] = r
    cz = out[(sy.SEC_Q_2NS, 0, 0)]
    q, xp = (0, 0, 0), (1, 0, 0)
    for piece in range(inst.q_deg):
        qp = _f3_mul(xp, evals[inst.ev_index[(sy.SEC_CM4_2NS, 3 * piece, 0)]])
        q = tuple((u + v) % P for u, v in zip(q, qp))
        xp = _f3_mul(xp, xin)
    return cz, q


def verify(inst, proof, verkey, publics, low_degree=True):
    """All checks of the module doc on a zkin-layout proof (canonical strings
    or ints; the final-degree check only with low_degree).  Returns the
    mismatch counters; every one 0 = the proof passes."""
    from oracle import oracle as oc
    steps = list(inst.fri_steps)
    pub = [int(v) for v in publics]
    bad, ys, ch = gr.verify_fri(oc, proof, [int(v) for v in verkey], pub, steps, inst.n_queries)
    f = fri_pol_at_rows(oc, inst, proof, ys, ch, pub)
    bad["fri_pol"] = 0
    if len(steps) > 1:
        w = 3 << (steps[0] - steps[1])
        s1 = _a2(proof["s1_vals"], w)
        for q, y in enumerate(ys):
            k = y >> steps[1]
            if not np.array_equal(f[q], s1[q, 3 * k:3 * k + 3]):
                bad["fri_pol"] += 1
    if low_degree:
        bad["final_degree"] = final_degree_ok(oc, inst, proof)[1]
        cz, q = quotient_identity(inst, proof, ch, pub)
        bad["quotient_at_xi"] = int(cz != q)
    bad["queries"] = len(ys)
    return bad


def failures(bad):
    return {k: v for k, v in bad.items() if k not in ("checked", "queries") and v}
