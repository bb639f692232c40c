// Goldilocks field F_p (p = 2^64 - 2^32 + 1) and cubic extension F_p[x]/(x^3-x-1)
// for gfx950 device code.
//
// Semantics follow the reference's Goldilocks/Goldilocks3 API (submodule, used
// e.g. at polinomial.hpp:178-207): every function returns a canonical value
// (< p) given canonical inputs; loads from user buffers go through gl_canon so
// non-canonical u64 inputs are accepted like the reference does.
//
// CDNA4 has no 64x64 multiply: the product is built from four 32x32->64
// partial products (v_mad_u64_u32) and reduced with 2^64 = 2^32-1 (mod p),
// 2^96 = -1 (mod p).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ZK_P 0xFFFFFFFF00000001ULL
#define ZK_EPS 0xFFFFFFFFULL

namespace zk {

__device__ __forceinline__ uint64_t gl_canon(uint64_t a) { return a >= ZK_P ? a - ZK_P : a; }

__device__ __forceinline__ uint64_t gl_add(uint64_t a, uint64_t b)
{
    uint64_t s = a + b;
    s += (s < a) ? ZK_EPS : 0;
    return gl_canon(s);
}

__device__ __forceinline__ uint64_t gl_sub(uint64_t a, uint64_t b)
{
    uint64_t d = a - b;
    d -= (a < b) ? ZK_EPS : 0;
    return d;
}

__device__ __forceinline__ uint64_t gl_neg(uint64_t a) { return a ? ZK_P - a : 0; }

// (hi:lo) mod p, canonical
__device__ __forceinline__ uint64_t gl_reduce128(uint64_t lo, uint64_t hi)
{
    uint32_t hh = (uint32_t)(hi >> 32);
    uint32_t hl = (uint32_t)hi;
    uint64_t t0 = lo - hh;
    t0 -= (lo < hh) ? ZK_EPS : 0;
    uint64_t t1 = ((uint64_t)hl << 32) - hl;  // hl * (2^32 - 1)
    uint64_t r = t0 + t1;
    r += (r < t1) ? ZK_EPS : 0;
    return gl_canon(r);
}

__device__ __forceinline__ uint64_t gl_mul(uint64_t a, uint64_t b)
{
    uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    uint64_t p00 = (uint64_t)a0 * b0;
    uint64_t p01 = (uint64_t)a0 * b1;
    uint64_t p10 = (uint64_t)a1 * b0;
    uint64_t p11 = (uint64_t)a1 * b1;
    // mid = p01 + p10 (65 bits)
    uint64_t mid = p01 + p10;
    uint64_t mid_c = (mid < p01) ? 1ULL : 0ULL;
    uint64_t lo = p00 + (mid << 32);
    uint64_t lo_c = (lo < p00) ? 1ULL : 0ULL;
    uint64_t hi = p11 + (mid >> 32) + (mid_c << 32) + lo_c;
    return gl_reduce128(lo, hi);
}

__device__ __forceinline__ uint64_t gl_sqr(uint64_t a) { return gl_mul(a, a); }

__device__ __forceinline__ uint64_t gl_pow(uint64_t a, uint64_t e)
{
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = gl_mul(r, a);
        a = gl_mul(a, a);
        e >>= 1;
    }
    return r;
}

// x * m for a small constant m (< 2^32): two 32x32 products
__device__ __forceinline__ uint64_t gl_mul_small(uint64_t a, uint32_t m)
{
    uint64_t lo_p = (uint64_t)(uint32_t)a * m;
    uint64_t hi_p = (uint64_t)(uint32_t)(a >> 32) * m;  // < 2^64
    // a*m = lo_p + hi_p * 2^32
    uint64_t lo = lo_p + (hi_p << 32);
    uint64_t c = (lo < lo_p) ? 1ULL : 0ULL;
    uint64_t hi = (hi_p >> 32) + c;
    return gl_reduce128(lo, hi);
}

// ---------------------------------------------------------------- F_p^3
struct gl3 {
    uint64_t v[3];
};

__device__ __forceinline__ gl3 gl3_add(const gl3 &a, const gl3 &b)
{
    return gl3{{gl_add(a.v[0], b.v[0]), gl_add(a.v[1], b.v[1]), gl_add(a.v[2], b.v[2])}};
}

__device__ __forceinline__ gl3 gl3_sub(const gl3 &a, const gl3 &b)
{
    return gl3{{gl_sub(a.v[0], b.v[0]), gl_sub(a.v[1], b.v[1]), gl_sub(a.v[2], b.v[2])}};
}

__device__ __forceinline__ gl3 gl3_mul1(const gl3 &a, uint64_t b)
{
    return gl3{{gl_mul(a.v[0], b), gl_mul(a.v[1], b), gl_mul(a.v[2], b)}};
}

// polinomial.hpp:195-205 (Karatsuba over x^3 = x + 1)
__device__ __forceinline__ gl3 gl3_mul(const gl3 &a, const gl3 &b)
{
    uint64_t A = gl_mul(gl_add(a.v[0], a.v[1]), gl_add(b.v[0], b.v[1]));
    uint64_t B = gl_mul(gl_add(a.v[0], a.v[2]), gl_add(b.v[0], b.v[2]));
    uint64_t C = gl_mul(gl_add(a.v[1], a.v[2]), gl_add(b.v[1], b.v[2]));
    uint64_t D = gl_mul(a.v[0], b.v[0]);
    uint64_t E = gl_mul(a.v[1], b.v[1]);
    uint64_t F = gl_mul(a.v[2], b.v[2]);
    uint64_t G = gl_sub(D, E);
    gl3 r;
    r.v[0] = gl_sub(gl_add(C, G), F);
    r.v[1] = gl_sub(gl_sub(gl_sub(gl_add(A, C), E), E), D);
    r.v[2] = gl_sub(B, G);
    return r;
}

}  // namespace zk
