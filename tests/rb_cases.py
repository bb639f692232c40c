"""Inputs that force the rare corrections of the rare-branch field helpers.

csrc/gl_rb.hpp and gl_add_rb / gl_sub_rb (csrc/gl_device.hpp) take their
final correction behind a wave-uniform branch: the correction runs only when
some lane of the wave needs it, about 2^-32 of random operations.  This module
restates, in Python integers, the exact condition under which each helper's
device code takes that branch (`taken_*`), builds inputs that satisfy it
(`force_*`), and gives the big-integer value each helper must return (`ref`).
tests/test_rb_cases.py checks the constructions on the CPU; tests/test_gpu_rb.py
runs them through zkgpu_gl_field_selftest_rb_dev (include/zkgpu.h) on the GPU.
"""
P = 0xFFFFFFFF00000001
EPS = 0xFFFFFFFF
M64 = (1 << 64) - 1

# op numbers of zkgpu_gl_field_selftest_rb_dev
ADD, SUB, MUL, RED128, RED96S, DOTFIN, MUL2E_RB, MUL2E, POW7, SQR3, RED128_PLAIN, DOTFIN_PLAIN = range(12)


# ------------------------------------------------------------ branch conditions
def taken_add(a, b):
    s = a + b
    return s > M64 and (s - (1 << 64)) + EPS > M64


def taken_sub(a, b):
    return a < b and (a - b) % (1 << 64) < EPS


def taken_red128(lo, hi):
    return lo < (hi >> 32)


def taken_mul(a, b):
    pr = a * b
    return taken_red128(pr & M64, pr >> 64)


def taken_red96s(lo, hl):
    hl &= 0xFFFFFFFF
    return lo + hl * EPS > M64


def dot_words(a0, a1, a2):
    """Dot3::fin's (l2, h) for accumulators A0, A1, A2 (gl_device.hpp)."""
    l1 = a0 + ((a1 << 22) & M64)
    c1 = l1 >> 64
    l1 &= M64
    l2 = l1 + ((a2 << 43) & M64)
    c2 = l2 >> 64
    l2 &= M64
    h = (a1 >> 42) + (a2 >> 21) + c1 + c2
    return l2, h


def taken_dotfin(a0, a1, a2):
    l2, h = dot_words(a0, a1, a2)
    return taken_red128(l2, h)


def taken_mul2e(e, x):
    """mul2e_rb<e>'s rare correction (gl_rb.hpp; e = 0, 32, >= 96 and
    20 < e < 32 take mul2e's select form instead: the same condition, no
    branch)."""
    if e == 0 or e == 32 or e >= 96:
        return False
    if e < 32:
        hl = x >> (64 - e)
        return ((x << e) & M64) + hl * EPS > M64
    if e < 64:
        k = e - 32
        lo = (x << k) & M64
        hl = x >> (64 - k)
        l0, l1 = lo & 0xFFFFFFFF, lo >> 32
        s = l0 + l1
        u = ((s & 0xFFFFFFFF) << 32) | (0xFFFFFFFF if s >> 32 else 0)
        return u < l1 + hl
    k = e - 64
    lo = (x << k) & M64
    hl = (x >> (64 - k)) if k else 0
    l0, l1 = lo & 0xFFFFFFFF, lo >> 32
    a = (l0 - hl) & 0xFFFFFFFF
    c = l0 + l1 + (EPS if hl > l0 else 0)
    return (a << 32) < c


# ------------------------------------------------------------ values
def ref(op, a, b=0, c=0, e=0):
    if op == ADD:
        return (a + b) % P
    if op == SUB:
        return (a - b) % P
    if op == MUL:
        return a * b % P
    if op in (RED128, RED128_PLAIN):
        return (a + (b << 64)) % P
    if op == RED96S:
        return (a + ((b & 0xFFFFFFFF) << 64)) % P
    if op in (DOTFIN, DOTFIN_PLAIN):
        return (a + (b << 22) + (c << 43)) % P
    if op in (MUL2E_RB, MUL2E):
        return a * pow(2, e, P) % P
    if op == POW7:
        return pow(a, 7, P)
    if op == SQR3:
        return a * a % P
    raise ValueError(op)


# ------------------------------------------------------------ forcing inputs
def _r(rng, lo, hi):
    """uniform integer in [lo, hi]; rng = random.Random (big ints)"""
    return rng.randint(lo, hi)


def force_add(rng):
    # a + b >= 2^65 - EPS: both near 2^64 (non-canonical lazy values)
    a = _r(rng, (1 << 64) - (1 << 31), M64)
    b = _r(rng, (1 << 65) - EPS - a, M64)
    return a, b


def force_sub(rng):
    # b - a >= p
    a = _r(rng, 0, EPS - 1)
    b = _r(rng, a + P, M64)
    return a, b


def force_red128(rng):
    hi = _r(rng, 1 << 32, M64)
    lo = _r(rng, 0, (hi >> 32) - 1)
    return lo, hi


def force_mul(rng):
    """a * b with the low product word below the top 32 bits of the high
    word: a odd, b = a^-1 * t mod 2^64 (small t), so a*b = t mod 2^64."""
    while True:
        a = _r(rng, 1 << 40, M64) | 1
        t = _r(rng, 0, 1 << 20)
        b = pow(a, -1, 1 << 64) * t % (1 << 64)
        if taken_mul(a, b):
            return a, b


def force_red96s(rng):
    hl = _r(rng, 1, 0xFFFFFFFF)
    lo = _r(rng, (1 << 64) - hl * EPS, M64)
    return lo, hl


def force_dotfin(rng):
    """Accumulators whose 128-bit sum has a high word >= 2^32 and a tiny low
    word (A0 + A1 2^22 + A2 2^43 = T, T < 2^106)."""
    while True:
        H = _r(rng, 1 << 32, (1 << 41) - 1)
        L = _r(rng, 0, (H >> 32) - 1)
        T = (H << 64) + L
        # random split of T over the three weighted accumulators
        a2 = _r(rng, max(0, (T - (1 << 64) * (1 << 22)) >> 43), T >> 43)
        rem = T - (a2 << 43)
        a1 = _r(rng, max(0, -((M64 - rem) >> 22)), min(rem >> 22, M64))
        a0 = rem - (a1 << 22)
        if a0 <= M64 and a1 <= M64 and a2 <= M64 and taken_dotfin(a0, a1, a2):
            return a0, a1, a2


def force_mul2e(e, rng):
    """x with mul2e_rb<e>'s correction taken (1 <= e < 96, e != 32)."""
    if e < 32:
        hl = _r(rng, 1, (1 << e) - 1)
        r = _r(rng, 1, (hl * EPS) >> e) << e  # lo = 2^64 - r, low e bits zero
        lo = (1 << 64) - r
        return (hl << (64 - e)) | (lo >> e)
    if e < 64:
        k = e - 32
        return _r(rng, 1, (1 << k) - 1) << (64 - k)  # lo = 0, hl > 0
    k = e - 64
    if k == 0 or rng.random() < 0.5:
        return _r(rng, 1, 0xFFFFFFFF) << (32 - k)  # hl = 0, l0 = 0, l1 > 0
    # hl = 2^k - 1, l0 = 2^k, l1 > 2^32 - 2^k  (a = 1, c > 2^32)
    l1 = _r(rng, (1 << 32) - (1 << k) + 1, 0xFFFFFFFF)
    lo = (l1 << 32) | (1 << k)
    return (((1 << k) - 1) << (64 - k)) | (lo >> k)


SPECIAL = [0, 1, 2, P - 2, P - 1, P, P + 1, P + 2**31, M64 - 1, M64, 2**32 - 1, 2**32, 2**32 + 1, 2**63, 2**63 - 1,
           2**64 - 2**32, 2**64 - 2**32 - 1, 2**48, 0xFFFFFFFF00000000]


def ordinary(rng, n):
    """random lazy u64 (half of them in [p, 2^64)); rng = random.Random"""
    return [rng.randint(0, M64) if i % 2 == 0 else rng.randint(P, M64) for i in range(n)]


def force_sqr(rng):
    """x = m 2^32 (m >= 2^16): x^2 = m^2 2^64 has a zero low word and a
    non-zero top half of the high word (gl_sqr3's reduction corrects)"""
    return _r(rng, 1 << 16, 0xFFFFFFFF) << 32


def taken_sqr(x):
    return taken_red128((x * x) & M64, (x * x) >> 64)
