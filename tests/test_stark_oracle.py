"""The oracle's synthetic STARK prover produces VALID proofs.

Validity is checked like a verifier would: FRI layers consistent with their
Merkle roots and with the folds (golden_replay.verify_fri, the same code that
replays the reference's golden proofs), the final polynomial has degree
< 2^last / blowup, and the quotient identity C(xi) = Z_H(xi) * sum_p xi^(pN) q_p(xi)
holds at the transcript's xi using the proof's evals.
"""
import numpy as np
import pytest

from golden_replay import arr, verify_fri

P = 0xFFFFFFFF00000001


def make(n_bits=8, blow=1, t=4, m=2, n_k=3, q=8, seed=0x5EED, q_deg=2):
    from zkgpu.synthetic import SyntheticStark
    from oracle.stark_prover import OracleStark
    inst = SyntheticStark(n_bits=n_bits, blowup_bits=blow, t=t, m=m, n_k=n_k, n_queries=q, seed=seed, q_deg=q_deg)
    o = OracleStark(inst)
    o.witness()
    return inst, o, o.prove()


def e3(v):
    return [int(x) % P for x in v]


def m3(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    c = [0] * 5
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            c[i + j] += x * y
    c[2] += c[4]; c[1] += c[4]
    c[1] += c[3]; c[0] += c[3]
    return [v % P for v in c[:3]]


def add3(a, b): return [(x + y) % P for x, y in zip(a, b)]
def sub3(a, b): return [(x - y) % P for x, y in zip(a, b)]
def sc3(a, s): return [x * s % P for x in a]
def b3(x): return [int(x) % P, 0, 0]


def pow3(a, e):
    r = [1, 0, 0]
    while e:
        if e & 1:
            r = m3(r, a)
        a = m3(a, a)
        e >>= 1
    return r


def quotient_identity(inst, proof, ch):
    """C(xi) from the evals, Horner in alpha, vs Z_H(xi) * sum_p xi^(pN) q_p(xi)."""
    N = 1 << inst.n_bits
    ev = [e3(v) for v in proof["evals"]]
    E = lambda sec, c, pr=0: ev[inst.ev_index[(sec, c, pr)]]
    S = __import__("zkgpu.synthetic", fromlist=["x"])
    u, dv, gamma, beta, alpha, xi = (e3(ch[k]) for k in (0, 1, 2, 3, 4, 7))
    cons = []
    for j in range(inst.t):
        a0, a1, a2 = (E(S.SEC_CM1_2NS, 3 * j + k) for k in range(3))
        kk = E(S.SEC_CONST_2NS, j % inst.n_k)
        cons.append(sub3(a2, add3(m3(m3(a0, a1), kk), a0)))
    for j, grp in enumerate(inst.groups):
        h = m3(u, E(S.SEC_CM1_2NS, grp[-1]))
        for c in reversed(grp[:-1]):
            h = m3(add3(h, E(S.SEC_CM1_2NS, c)), u)
        h = add3(h, dv)
        cons.append(sub3(E(S.SEC_CM2_2NS, 3 * j), h))
    for j in range(inst.m):
        cons.append(m3(sub3(E(S.SEC_CM3_2NS, 3 * j), [1, 0, 0]), E(S.SEC_CONST_2NS, inst.l_first)))
    for j in range(inst.m):
        r = m3(m3(add3(E(S.SEC_CM2_2NS, 3 * j, 1), gamma), beta), E(S.SEC_CM3_2NS, 3 * j, 1))
        s = m3(m3(add3(E(S.SEC_CM2_2NS, 3 * j, 0), gamma), beta), E(S.SEC_CM3_2NS, 3 * j, 0))
        cons.append(sub3(r, s))
    if inst.with_step3:  # W - (Z_0 a_0 + K_0), W written by step3 after calculateZ
        w = add3(m3(E(S.SEC_CM3_2NS, inst.z_ctx[0][2]), E(S.SEC_CM1_2NS, 0)), E(S.SEC_CONST_2NS, 0))
        cons.append(sub3(E(S.SEC_CM3_2NS, inst.cm3_w), w))
    # plookups (pil-stark Plookup): L_first (Z - 1); Z' den - Z num
    one = [1, 0, 0]
    ob = add3(beta, one)
    gb = m3(ob, gamma)
    for k, lk in enumerate(inst.lookups):
        cons.append(m3(sub3(E(S.SEC_CM3_2NS, lk["z"]), one), E(S.SEC_CONST_2NS, inst.l_first)))
        d = lk["dim"]
        if d == 3:
            f = add3(E(S.SEC_CM1_2NS, inst.cm1_lk[0]), m3(u, E(S.SEC_CM1_2NS, inst.cm1_lk[1])))
            t = add3(E(S.SEC_CONST_2NS, inst.c_t[0]), m3(u, E(S.SEC_CONST_2NS, inst.c_t[1])))
            tn = add3(E(S.SEC_CONST_2NS, inst.c_t[0], 1), m3(u, E(S.SEC_CONST_2NS, inst.c_t[1], 1)))
        else:
            f = E(S.SEC_CM1_2NS, inst.cm1_lk[2])
            t = E(S.SEC_CONST_2NS, inst.c_t[2])
            tn = E(S.SEC_CONST_2NS, inst.c_t[2], 1)
        h1, h2 = E(S.SEC_CM2_2NS, lk["h1"]), E(S.SEC_CM2_2NS, lk["h2"])
        h1n = E(S.SEC_CM2_2NS, lk["h1"], 1)
        num = m3(m3(ob, add3(f, gamma)), add3(add3(gb, t), m3(beta, tn)))
        den = m3(add3(add3(gb, h1), m3(beta, h2)), add3(add3(gb, h2), m3(beta, h1n)))
        z, zn = E(S.SEC_CM3_2NS, lk["z"]), E(S.SEC_CM3_2NS, lk["z"], 1)
        cons.append(sub3(m3(zn, den), m3(z, num)))
    C = cons[0]
    for c in cons[1:]:
        C = add3(m3(C, alpha), c)
    zh = sub3(pow3(xi, N), [1, 0, 0])
    xiN = pow3(xi, N)
    acc = [0, 0, 0]
    cur = [1, 0, 0]
    for p in range(inst.q_deg):
        acc = add3(acc, m3(cur, E(S.SEC_CM4_2NS, 3 * p)))
        cur = m3(cur, xiN)
    return C == m3(zh, acc)


@pytest.mark.parametrize("n_bits,blow,t,m,q_deg", [(8, 1, 4, 2, 2), (9, 2, 3, 1, 2), (10, 1, 6, 3, 2),
                                                   (8, 2, 3, 2, 4), (8, 3, 2, 1, 5)])
def test_synthetic_proof_is_valid(oracle, n_bits, blow, t, m, q_deg):
    """q_deg > 2 (blowup 2^2, 2^3): the quotient split writes q_deg pieces,
    the ones above the constraint degree are zero polynomials."""
    inst, o, proof = make(n_bits=n_bits, blow=blow, t=t, m=m, q_deg=q_deg)
    bad, ys, ch = verify_fri(oracle, proof, o.verkey, o.publics, inst.fri_steps, inst.n_queries)
    assert bad["s0"] == 0 and bad["fri_tree"] == 0 and bad["fold"] == 0 and bad["final"] == 0, bad
    # challenges re-derived by the verifier equal the prover's
    for k in (0, 1, 2, 3, 4, 5, 6, 7):
        assert np.array_equal(ch[k], o.challenges[k])
    # final polynomial: degree < 2^last / blowup (values on a coset -> interpolate)
    fp = arr(proof["finalPol"]).reshape(-1, 3)
    coef = oracle.ntt(fp, True)
    deg_bound = (1 << inst.fri_steps[-1]) >> blow
    assert not coef[deg_bound:].any()
    assert coef[:deg_bound].any()
    assert quotient_identity(inst, proof, ch)


def test_tampered_trace_breaks_validity(oracle):
    """Negative control: an invalid witness gives a proof the checks reject."""
    from zkgpu.synthetic import SyntheticStark
    from oracle.stark_prover import OracleStark
    inst = SyntheticStark(n_bits=8, blowup_bits=1, t=4, m=2, n_queries=8)
    o = OracleStark(inst)
    o.witness()
    o.S[0][17, 2] ^= 1  # break a[2] = a[0]*a[1]*K + a[0] at one row
    proof = o.prove()
    bad, ys, ch = verify_fri(oracle, proof, o.verkey, o.publics, inst.fri_steps, inst.n_queries)
    fp = arr(proof["finalPol"]).reshape(-1, 3)
    coef = oracle.ntt(fp, True)
    deg_bound = (1 << inst.fri_steps[-1]) >> 1
    assert coef[deg_bound:].any() or not quotient_identity(inst, proof, ch)


def test_lookup_value_not_in_table_is_rejected(oracle):
    """calculateH1H2 refuses an f value absent from the table ("Number not
    included", polinomial.hpp:409-413), like the reference."""
    from zkgpu.synthetic import SyntheticStark
    from oracle.stark_prover import OracleStark
    inst = SyntheticStark(n_bits=8, blowup_bits=1, t=4, m=2, n_queries=8)
    o = OracleStark(inst)
    o.witness()
    o.S[0][9, inst.cm1_lk[2]] = 12345  # not a T2 value
    with pytest.raises(ValueError, match="Number not included: w=9"):
        o.prove()
