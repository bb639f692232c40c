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
Not checked: the constraint identity C(xi) Z_H(xi)^-1 = sum_p xi^(pN) q_p(xi),
which needs the verifier's evaluation of step42ns at an extension-field point
(the oracle interpreter evaluates on base-field domain points only) and, for
the zkEVM-shaped instance, a trace that satisfies its constraints (it does
not: the quotient there is not a low-degree polynomial).
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
    bad["queries"] = len(ys)
    return bad


def failures(bad):
    return {k: v for k, v in bad.items() if k not in ("checked", "queries") and v}
