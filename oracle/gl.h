/*
 * oracle/gl.h -- TEST INFRASTRUCTURE ONLY (CPU oracle, never shipped, never
 * on the product path).  Goldilocks field F_p, p = 2^64 - 2^32 + 1, and its
 * cubic extension F_p[x]/(x^3 - x - 1).
 *
 * Restates the semantics the reference takes from the absent submodule
 * `src/goldilocks` (goldilocks_base_field.hpp / goldilocks_cubic_extension.hpp,
 * see .gitmodules:1-3):
 *   - every result is returned canonical (< p); inputs may be any u64;
 *   - Goldilocks::w(n) = W[n] = W32^(2^(32-n)), W32 = 7277203076849721926
 *     (value pinned against the golden proofs);
 *   - Goldilocks::shift() = 7;
 *   - cubic multiplication exactly as polinomial.hpp:195-205 (Karatsuba form).
 */
#ifndef ORACLE_GL_H
#define ORACLE_GL_H

#include <stdint.h>

#define GL_P 0xFFFFFFFF00000001ULL
#define GL_EPS 0xFFFFFFFFULL /* 2^64 mod p */
#define GL_W32 7277203076849721926ULL
#define GL_SHIFT 7ULL

typedef unsigned __int128 u128;

static inline uint64_t gl_canon(uint64_t a) { return a >= GL_P ? a - GL_P : a; }

static inline uint64_t gl_add(uint64_t a, uint64_t b)
{
    a = gl_canon(a);
    b = gl_canon(b);
    uint64_t s = a + b;
    /* a,b < p so a+b < 2p < 2^65; overflow past 2^64 means s + 2^64 - p */
    if (s < a) s += GL_EPS;
    return gl_canon(s);
}

static inline uint64_t gl_sub(uint64_t a, uint64_t b)
{
    a = gl_canon(a);
    b = gl_canon(b);
    return a >= b ? a - b : a + (GL_P - b);
}

static inline uint64_t gl_neg(uint64_t a)
{
    a = gl_canon(a);
    return a ? GL_P - a : 0;
}

/* reduce a 128-bit value mod p (2^64 = eps, 2^96 = -1) */
static inline uint64_t gl_reduce128(u128 x)
{
    uint64_t lo = (uint64_t)x;
    uint64_t hi = (uint64_t)(x >> 64);
    uint64_t hi_hi = hi >> 32;
    uint64_t hi_lo = hi & GL_EPS;
    uint64_t t0 = lo - hi_hi;
    if (lo < hi_hi) t0 -= GL_EPS; /* borrow: t0 += p, i.e. -= eps mod 2^64 */
    uint64_t t1 = hi_lo * GL_EPS;
    uint64_t r = t0 + t1;
    if (r < t0) r += GL_EPS;
    return gl_canon(r);
}

static inline uint64_t gl_mul(uint64_t a, uint64_t b) { return gl_reduce128((u128)a * b); }

static inline uint64_t gl_pow(uint64_t a, uint64_t e)
{
    uint64_t r = 1;
    a = gl_canon(a);
    while (e) {
        if (e & 1) r = gl_mul(r, a);
        a = gl_mul(a, a);
        e >>= 1;
    }
    return r;
}

static inline uint64_t gl_inv(uint64_t a) { return gl_pow(a, GL_P - 2); }

/* W[n]: primitive 2^n-th root of unity used by the reference (n <= 32) */
static inline uint64_t gl_w(unsigned n)
{
    uint64_t w = GL_W32;
    for (unsigned i = n; i < 32; i++) w = gl_mul(w, w);
    return w;
}

/* ---------------- cubic extension, element = 3 consecutive u64 ---------- */
static inline void gl3_add(uint64_t *o, const uint64_t *a, const uint64_t *b)
{
    o[0] = gl_add(a[0], b[0]);
    o[1] = gl_add(a[1], b[1]);
    o[2] = gl_add(a[2], b[2]);
}

static inline void gl3_sub(uint64_t *o, const uint64_t *a, const uint64_t *b)
{
    o[0] = gl_sub(a[0], b[0]);
    o[1] = gl_sub(a[1], b[1]);
    o[2] = gl_sub(a[2], b[2]);
}

static inline void gl3_mul1(uint64_t *o, const uint64_t *a, uint64_t b)
{
    o[0] = gl_mul(a[0], b);
    o[1] = gl_mul(a[1], b);
    o[2] = gl_mul(a[2], b);
}

/* polinomial.hpp:195-205 */
static inline void gl3_mul(uint64_t *o, const uint64_t *a, const uint64_t *b)
{
    uint64_t A = gl_mul(gl_add(a[0], a[1]), gl_add(b[0], b[1]));
    uint64_t B = gl_mul(gl_add(a[0], a[2]), gl_add(b[0], b[2]));
    uint64_t C = gl_mul(gl_add(a[1], a[2]), gl_add(b[1], b[2]));
    uint64_t D = gl_mul(a[0], b[0]);
    uint64_t E = gl_mul(a[1], b[1]);
    uint64_t F = gl_mul(a[2], b[2]);
    uint64_t G = gl_sub(D, E);
    uint64_t r0 = gl_sub(gl_add(C, G), F);
    uint64_t r1 = gl_sub(gl_sub(gl_sub(gl_add(A, C), E), E), D);
    uint64_t r2 = gl_sub(B, G);
    o[0] = r0;
    o[1] = r1;
    o[2] = r2;
}

/* inverse in F_p^3 by a^(p^3-2) */
static inline void gl3_inv(uint64_t *o, const uint64_t *a)
{
    /* e = p^3 - 2 as 192-bit little-endian limbs */
    u128 p2 = (u128)GL_P * GL_P;
    /* p^3 = p2 * p: compute as 3 limbs */
    uint64_t l0, l1, l2;
    {
        u128 lo = (u128)(uint64_t)p2 * GL_P;
        u128 hi = (u128)(uint64_t)(p2 >> 64) * GL_P;
        l0 = (uint64_t)lo;
        u128 mid = (lo >> 64) + (uint64_t)hi;
        l1 = (uint64_t)mid;
        l2 = (uint64_t)(hi >> 64) + (uint64_t)(mid >> 64);
    }
    /* subtract 2 */
    if (l0 >= 2) {
        l0 -= 2;
    } else {
        l0 -= 2;
        if (l1-- == 0) l2--;
    }
    uint64_t limbs[3] = {l0, l1, l2};
    uint64_t r[3] = {1, 0, 0};
    uint64_t base[3] = {gl_canon(a[0]), gl_canon(a[1]), gl_canon(a[2])};
    for (int li = 0; li < 3; li++) {
        uint64_t e = limbs[li];
        for (int bit = 0; bit < 64; bit++) {
            if (e & 1) gl3_mul(r, r, base);
            gl3_mul(base, base, base);
            e >>= 1;
        }
    }
    o[0] = r[0];
    o[1] = r[1];
    o[2] = r[2];
}

#endif /* ORACLE_GL_H */
