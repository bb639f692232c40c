"""Rare-branch field helpers on the GPU vs big integers.

csrc/gl_rb.hpp's helpers and gl_add_rb / gl_sub_rb take their final
correction only when the wave's ballot of it is non-zero -- about 2^-32 of
random operations, so random-input parity tests almost never reach it.  Each
op here runs through zkgpu_gl_field_selftest_rb_dev on inputs built to force
the correction (tests/rb_cases.py, checked on the CPU by test_rb_cases.py):
(a) in every lane of a wave, (b) in exactly one lane of an otherwise ordinary
wave, (c) the edge values pairwise; outputs are compared with big integers.
Then one radix-256 NTT pass chain (forward, inverse, LDE) whose first
butterfly stage sees a forced second carry / borrow, against the oracle.
Reference semantics: the Goldilocks field ops of starks.cpp:53.
"""
import random

import numpy as np
import pytest

import rb_cases as rc

pytestmark = pytest.mark.gpu

WAVES = 4


def _layouts(force, rng, n_ord_waves=WAVES):
    """(inputs, forced mask): 4 waves all forced, then 4 ordinary waves with
    one forced lane each (lane 0, 63 and two random ones)"""
    rows, forced = [], []
    for _ in range(64 * WAVES):
        rows.append(force(rng))
        forced.append(True)
    lanes = [0, 63, rng.randrange(1, 63), rng.randrange(1, 63)]
    for w in range(n_ord_waves):
        for lane in range(64):
            if lane == lanes[w]:
                rows.append(force(rng))
                forced.append(True)
            else:
                rows.append(tuple(rc.ordinary(rng, 3)))
                forced.append(False)
    return rows, forced


def _run(zkgpu, op, rows, e=0):
    import torch
    n = len(rows)
    cols = list(zip(*[(r + (0, 0))[:3] for r in rows]))
    a, b, c = (np.array(col, dtype=np.uint64) for col in cols)
    out = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    zkgpu.field_selftest_rb_dev(out, zkgpu.to_device(a), zkgpu.to_device(b), zkgpu.to_device(c), n, op, e)
    torch.cuda.synchronize()
    got = zkgpu.from_device(out)
    exp = [rc.ref(op, *((r + (0, 0))[:3]), e=e) for r in rows]
    bad = [i for i in range(n) if int(got[i]) != exp[i]]
    assert not bad, [(i, [hex(v) for v in rows[i]], hex(int(got[i])), hex(exp[i])) for i in bad[:5]]


CASES = {
    "add": (rc.ADD, lambda g: rc.force_add(g), rc.taken_add),
    "sub": (rc.SUB, lambda g: rc.force_sub(g), rc.taken_sub),
    "mul": (rc.MUL, lambda g: rc.force_mul(g), rc.taken_mul),
    "reduce128": (rc.RED128, lambda g: rc.force_red128(g), rc.taken_red128),
    "reduce128_plain": (rc.RED128_PLAIN, lambda g: rc.force_red128(g), rc.taken_red128),
    "reduce96_small": (rc.RED96S, lambda g: rc.force_red96s(g), rc.taken_red96s),
    "dot3_fin": (rc.DOTFIN, lambda g: rc.force_dotfin(g), rc.taken_dotfin),
    "dot3_fin_plain": (rc.DOTFIN_PLAIN, lambda g: rc.force_dotfin(g), rc.taken_dotfin),
    "sqr3": (rc.SQR3, lambda g: (rc.force_sqr(g),), rc.taken_sqr),
    "pow7": (rc.POW7, lambda g: (rc.force_sqr(g),), rc.taken_sqr),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_rb_helper_forced(zkgpu, name):
    op, force, taken = CASES[name]
    rng = random.Random(name)
    rows, forced = _layouts(force, rng)
    assert all(taken(*r) for r, f in zip(rows, forced) if f)
    _run(zkgpu, op, rows)


@pytest.mark.parametrize("name", sorted(CASES))
def test_rb_helper_edges(zkgpu, name):
    op = CASES[name][0]
    sp = rc.SPECIAL
    rows = [(x, y, (x ^ y) >> 1) for x in sp for y in sp]
    _run(zkgpu, op, rows)


@pytest.mark.parametrize("op", [rc.MUL2E_RB, rc.MUL2E], ids=["mul2e_rb", "mul2e"])
def test_mul2e_every_exponent(zkgpu, op):
    """every E in [0, 192): forced corrections (where mul2e_rb<E> has one) in
    all lanes and in one lane, then edge and random values"""
    for e in range(192):
        rng = random.Random(1000 * op + e)
        if 0 < e < 96 and e != 32:
            rows, forced = _layouts(lambda g: (rc.force_mul2e(e, g),), rng, 2)
            assert all(rc.taken_mul2e(e, r[0]) for r, f in zip(rows, forced) if f)
        else:
            rows = [(x,) for x in rc.ordinary(rng, 128)]
        rows += [(x,) for x in rc.SPECIAL]
        _run(zkgpu, op, rows, e)


# ------------------------------------------------------------------ NTT pass chain
M = rc.M64


def _ntt_inputs(n, rng):
    """column 0: every lane adversarial (values drawn from {0, 2^64-1,
    2^64-2, p, p+1}); column 1: canonical random with forced pairs at
    (i, i + n/2) -- the first radix-256 butterfly stage's operands --
    (2^64-1, 2^64-1) forcing the add's second carry, (0, 2^64-1) the forward
    difference's second borrow and (2^64-1, 0) the inverse's"""
    x = np.empty((n, 2), np.uint64)
    pool = np.array([0, M, M - 1, rc.P, rc.P + 1], dtype=np.uint64)
    x[:, 0] = pool[np.array([rng.randrange(5) for _ in range(n)])]
    x[:, 1] = np.array([rng.randrange(rc.P) for _ in range(n)], dtype=np.uint64)
    h = n // 2
    for i, (u, v) in zip(rng.sample(range(h), 3), [(M, M), (0, M), (M, 0)]):
        x[i, 1], x[i + h, 1] = u, v
    assert rc.taken_add(M, M) and rc.taken_sub(0, M)
    return x


@pytest.mark.parametrize("logn", [16, 20])
@pytest.mark.parametrize("inverse", [False, True])
def test_ntt_pass_forced_second_carry(oracle, zkgpu, logn, inverse):
    rng = random.Random(logn * 2 + inverse)
    x = _ntt_inputs(1 << logn, rng)
    got = zkgpu.ntt(x, inverse=inverse)
    exp = oracle.ntt(x % np.uint64(rc.P), inverse=inverse)
    assert np.array_equal(got, exp)


def test_lde_forced_second_carry(oracle, zkgpu):
    rng = random.Random(5)
    n = 1 << 18
    x = _ntt_inputs(n, rng)
    got = zkgpu.extend_pol(x, 2 * n)
    exp = oracle.extend_pol(x % np.uint64(rc.P), 2 * n)
    assert np.array_equal(got, exp)
