"""CPU checks of the rare-branch forcing inputs (tests/rb_cases.py): every
constructed input takes its helper's correction, and the reference values
agree with an independent restatement of the device arithmetic."""
import random

import pytest

import rb_cases as rc


@pytest.mark.parametrize("name", ["add", "sub", "red128", "mul", "red96s", "dotfin"])
def test_forcing_inputs_take_the_branch(name):
    rng = random.Random(name)
    force = getattr(rc, "force_" + name)
    taken = getattr(rc, "taken_" + name)
    for _ in range(200):
        assert taken(*force(rng))


@pytest.mark.parametrize("e", [e for e in range(1, 96) if e != 32])
def test_forcing_inputs_mul2e(e):
    rng = random.Random(e)
    for _ in range(50):
        x = rc.force_mul2e(e, rng)
        assert 0 <= x <= rc.M64 and rc.taken_mul2e(e, x), (e, hex(x))


def test_random_inputs_rarely_take_the_branch():
    # uniform u64 (values >= p in both operands of an add do reach it: the
    # GPU tests place those too)
    rng = random.Random(7)
    xs = [rng.randint(0, rc.M64) for _ in range(4000)]
    ys = [rng.randint(0, rc.M64) for _ in range(4000)]
    assert sum(rc.taken_add(a, b) or rc.taken_sub(a, b) or rc.taken_mul(a, b) for a, b in zip(xs, ys)) == 0


def _dot_fin_model(a0, a1, a2):
    """Dot3::fin + gl_reduce128 in 64-bit words (gl_device.hpp)."""
    l2, h = rc.dot_words(a0, a1, a2)
    hh, hl = h >> 32, h & 0xFFFFFFFF
    t0 = (l2 - hh) % (1 << 64)
    if l2 < hh:
        t0 = (t0 - rc.EPS) % (1 << 64)
    t1 = ((hl << 32) - hl) % (1 << 64)
    r = t0 + t1
    if r > rc.M64:
        r = (r - (1 << 64)) + rc.EPS
    return r


def test_dot_fin_model_matches_reference():
    rng = random.Random(3)
    for _ in range(300):
        a = rc.force_dotfin(rng)
        assert _dot_fin_model(*a) % rc.P == rc.ref(rc.DOTFIN, *a)
    for _ in range(300):
        a = [rng.randint(0, 2**63) for _ in range(3)]
        assert _dot_fin_model(*a) % rc.P == rc.ref(rc.DOTFIN, *a)
