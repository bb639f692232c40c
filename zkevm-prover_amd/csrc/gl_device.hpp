// Goldilocks field F_p (p = 2^64 - 2^32 + 1) and cubic extension F_p[x]/(x^3-x-1)
// for gfx950 device code.
//
// Representation: "lazy".  Every operation accepts ANY u64 as an element
// (value = x mod p) and returns some u64 congruent to the result -- not
// necessarily < p.  Kernels canonicalise exactly once, with gl_canon() on
// every store to a user-visible buffer (outputs are canonical, like the
// reference's toU64/toString), and before any comparison of values.
// Measured on MI355X (tools/microbench.hip): the lazy multiply runs 1.6x
// faster than one that canonicalises every product.
//
// CDNA4 has no 64x64 multiply: the 128-bit product is built from four
// 32x32->64 multiply-adds (v_mad_u64_u32) and folded with
// 2^64 = 2^32 - 1 (mod p) and 2^96 = -1 (mod p).
//
// Semantics match the reference's Goldilocks/Goldilocks3 API (submodule,
// used e.g. at polinomial.hpp:178-207) after canonicalisation.
#ifndef __HIPCC_RTC__
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#else
// run-time compiled expression kernels (csrc/zxp_jit.hip) embed this file
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
using __hip_internal::int64_t;
using __hip_internal::int32_t;
#endif

#define ZK_P 0xFFFFFFFF00000001ULL
#define ZK_EPS 0xFFFFFFFFULL  // 2^64 mod p

namespace zk {

// Accesses through a pointer that was itself read from memory (column tables,
// term records): the compiler cannot infer the global address space there and
// emits FLAT instructions, which also count against LGKM_CNT -- every
// s_waitcnt for a scalar constant load would then wait for them as well.
typedef __attribute__((address_space(1))) uint64_t gu64_t;
__device__ __forceinline__ uint64_t gload(const uint64_t *p) { return *(const gu64_t *)p; }
__device__ __forceinline__ void gstore(uint64_t *p, uint64_t v) { *(gu64_t *)p = v; }
// A store to a column the same kernel never loads (the expression kernels'
// output / carry columns, csrc/zxp_jit.hip): written as a double, a type no
// load of the kernel uses, so type-based alias analysis lets the scheduler
// move column loads across it.  The bits are the u64's.
typedef __attribute__((address_space(1))) double gf64_t;
__device__ __forceinline__ void gstore_out(uint64_t *p, uint64_t v) { *(gf64_t *)p = __builtin_bit_cast(double, v); }

// any u64 -> [0, p)   (x < 2^64 < 2p, so one conditional subtraction)
__device__ __forceinline__ uint64_t gl_canon(uint64_t a) { return a >= ZK_P ? a - ZK_P : a; }

// ZK_RB = 1 (a translation unit's choice, e.g. a run-time compiled
// expression kernel): gl_add / gl_sub take the rare second correction behind
// a wave-uniform branch, as gl_add_rb / gl_sub_rb below
#ifndef ZK_RB
#define ZK_RB 0
#endif

// a + b (mod p), any inputs, lazy output
__device__ __forceinline__ uint64_t gl_add(uint64_t a, uint64_t b)
{
    uint64_t s, s2;
    bool c = __builtin_add_overflow(a, b, &s);  // a + b = s + 2^64 c  ==  s + EPS c
    bool c2 = __builtin_add_overflow(s, c ? ZK_EPS : 0ULL, &s2);
#if ZK_RB
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(c2) != 0, 0)) s2 += c2 ? ZK_EPS : 0ULL;
    return s2;
#else
    return s2 + (c2 ? ZK_EPS : 0ULL);  // c2 => s2 < EPS: no third carry
#endif
}

// a - b (mod p), any inputs, lazy output
__device__ __forceinline__ uint64_t gl_sub(uint64_t a, uint64_t b)
{
    uint64_t d, d2;
    bool br = __builtin_sub_overflow(a, b, &d);  // a - b = d - 2^64 br  ==  d - EPS br
    bool br2 = __builtin_sub_overflow(d, br ? ZK_EPS : 0ULL, &d2);
#if ZK_RB
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(br2) != 0, 0)) d2 -= br2 ? ZK_EPS : 0ULL;
    return d2;
#else
    return d2 - (br2 ? ZK_EPS : 0ULL);  // br2 => d2 > 2^64 - EPS: no third borrow
#endif
}

__device__ __forceinline__ uint64_t gl_neg(uint64_t a) { return gl_sub(0, a); }

// gl_add / gl_sub with the second correction behind a wave-uniform branch.
// The second carry (borrow) needs a + b - 2^64 >= 2^64 - EPS (b - a >= p):
// about 2^-32 per operation on lazy values, so a wave almost never takes
// it; the ballot is the compare's own lane mask, the branch is scalar, and
// the common path saves the select and the 64-bit add.  Same values as
// gl_add / gl_sub, bit for bit.
__device__ __forceinline__ uint64_t gl_add_rb(uint64_t a, uint64_t b)
{
    uint64_t s, s2;
    const bool c = __builtin_add_overflow(a, b, &s);
    const bool c2 = __builtin_add_overflow(s, c ? ZK_EPS : 0ULL, &s2);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(c2) != 0, 0)) s2 += c2 ? ZK_EPS : 0ULL;
    return s2;
}

__device__ __forceinline__ uint64_t gl_sub_rb(uint64_t a, uint64_t b)
{
    uint64_t d, d2;
    const bool br = __builtin_sub_overflow(a, b, &d);
    const bool br2 = __builtin_sub_overflow(d, br ? ZK_EPS : 0ULL, &d2);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(br2) != 0, 0)) d2 -= br2 ? ZK_EPS : 0ULL;
    return d2;
}

// (hi:lo) mod p, lazy output.  hi*2^64 = hh*2^96 + hl*2^64 == -hh + hl*EPS
__device__ __forceinline__ uint64_t gl_reduce128(uint64_t lo, uint64_t hi)
{
    const uint32_t hh = (uint32_t)(hi >> 32);
    const uint32_t hl = (uint32_t)hi;
    uint64_t t0, r;
    bool br = __builtin_sub_overflow(lo, (uint64_t)hh, &t0);
#if ZK_RB  // (br needs lo < hh < 2^32: rare)
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(br) != 0, 0)) t0 -= br ? ZK_EPS : 0ULL;
#else
    t0 -= br ? ZK_EPS : 0ULL;  // br => t0 >= 2^64 - 2^32 + 1 > EPS
#endif
    const uint64_t t1 = ((uint64_t)hl << 32) - hl;  // hl * EPS, <= 2^64 - 2^33 + 1
    bool c = __builtin_add_overflow(t0, t1, &r);
    return r + (c ? ZK_EPS : 0ULL);  // c => r < t1: no second carry
}

// lo + hl*2^64 for hl < 2^32 (no 2^96 term)
__device__ __forceinline__ uint64_t gl_reduce96(uint64_t lo, uint32_t hl)
{
    const uint64_t t1 = ((uint64_t)hl << 32) - hl;
    uint64_t r;
    bool c = __builtin_add_overflow(lo, t1, &r);
    return r + (c ? ZK_EPS : 0ULL);
}

__device__ __forceinline__ uint64_t gl_mul(uint64_t a, uint64_t b)
{
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);          // < 2^64
    const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;          // < 2^64
    const uint64_t hi = (uint64_t)a1 * b1 + (t >> 32) + (u >> 32);  // < 2^64
    const uint64_t lo = (u << 32) | (uint32_t)p00;
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

// x * 2^E (mod p), compile-time E in [0, 192): 2^96 = -1, 2^192 = 1.
// With lo = x << k = l0 + 2^32 l1 and hl = x >> (64 - k) (x 2^k = lo + 2^64 hl):
//   E = 32 + k (0 < k < 32):  x 2^E == (l0 + l1) 2^32 - (l1 + hl)
//   E = 64 + k (0 <= k < 32): x 2^E == (l0 - hl) 2^32 - (l0 + l1)
// (2^64 == 2^32 - 1, 2^96 == -1): 10-11 instructions instead of a 128-bit
// reduction (E < 64) or two chained shift-multiplies (E >= 64, 23-30).
template <int E>
__device__ __forceinline__ uint64_t mul2e(uint64_t x)
{
    static_assert(E >= 0 && E < 192, "exponent range");
    if constexpr (E == 0) {
        return x;
    } else if constexpr (E >= 96) {
        return gl_neg(mul2e<E - 96>(x));
    } else if constexpr (E <= 32) {
        return gl_reduce96(x << E, (uint32_t)(x >> (64 - E)));
    } else if constexpr (E < 64) {
        constexpr int k = E - 32;
        const uint64_t lo = x << k;
        const uint32_t hl = (uint32_t)(x >> (64 - k));
        const uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32);
        uint32_t s1;
        const uint32_t s0 = __builtin_addc(l0, l1, 0u, &s1);
        // (l0 + l1) 2^32 == s0 2^32 + s1 (2^32 - 1), < 2^64 as one word pair
        const uint64_t u = ((uint64_t)s0 << 32) | (s1 ? 0xFFFFFFFFu : 0u);
        uint64_t r;
        const bool b = __builtin_sub_overflow(u, (uint64_t)l1 + hl, &r);
        return r - (b ? ZK_EPS : 0ULL);  // b => r >= 2^64 - 2^33: no second borrow
    } else {
        constexpr int k = E - 64;
        const uint64_t lo = x << k;
        const uint32_t hl = k ? (uint32_t)(x >> (64 - (k ? k : 1))) : 0u;
        const uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32);
        // (l0 - hl) 2^32: when hl > l0, (2^32 + l0 - hl) 2^32 - 2^64 == ... - (2^32 - 1)
        const uint32_t a = l0 - hl;
        const uint64_t c = (uint64_t)l0 + l1 + (hl > l0 ? ZK_EPS : 0ULL);  // < 2^34
        uint64_t r;
        const bool b = __builtin_sub_overflow((uint64_t)a << 32, c, &r);
        return r - (b ? ZK_EPS : 0ULL);
    }
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

__device__ __forceinline__ gl3 gl3_canon(const gl3 &a)
{
    return gl3{{gl_canon(a.v[0]), gl_canon(a.v[1]), gl_canon(a.v[2])}};
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

// F_p^3 op F_p (the base operand sits in component 0)
__device__ __forceinline__ gl3 gl3_add1(const gl3 &a, uint64_t b) { return gl3{{gl_add(a.v[0], b), a.v[1], a.v[2]}}; }
__device__ __forceinline__ gl3 gl3_sub1(const gl3 &a, uint64_t b) { return gl3{{gl_sub(a.v[0], b), a.v[1], a.v[2]}}; }
__device__ __forceinline__ gl3 gl3_rsub1(uint64_t a, const gl3 &b)
{
    return gl3{{gl_sub(a, b.v[0]), gl_neg(b.v[1]), gl_neg(b.v[2])}};
}

// ---------------------------------------------------------------- dot products
// Dot product of lazy lanes with table coefficients, one reduction at the end.
// Coefficient c is stored as 22/21/21-bit limbs of c and of c*2^32 mod p
// (tools/gen_poseidon_sparse.py limbs6; api.hip zxp_limbs6 for ZXP_DOT), so
// a = a0 + a1*2^32 contributes a0*c_k + a1*c'_k to accumulator k (weights
// 2^0, 2^22, 2^43): six carry-free 32x32->64 multiply-adds per term, each
// term adding < 2^55 (< 2^61 for <= 34 terms, < 2^63 for <= 250).
struct alignas(16) LimbQ {
    uint32_t x, y, z, w;
};
struct alignas(8) LimbP {
    uint32_t x, y;
};

struct Dot3 {
    uint64_t A0, A1, A2;
    __device__ __forceinline__ explicit Dot3(const uint32_t *k) : A0(k[0]), A1(k[1]), A2(k[2]) {}
    __device__ __forceinline__ Dot3() : A0(0), A1(0), A2(0) {}
    // limbs of a ROW-VARYING coefficient c (any u64): c and c * 2^32 mod p
    __device__ __forceinline__ static void limbs(uint64_t c, uint32_t out[6])
    {
        const uint64_t cs = mul2e<32>(c);
        out[0] = (uint32_t)c & 0x3FFFFFu;
        out[1] = (uint32_t)(c >> 22) & 0x1FFFFFu;
        out[2] = (uint32_t)(c >> 43);
        out[3] = (uint32_t)cs & 0x3FFFFFu;
        out[4] = (uint32_t)(cs >> 22) & 0x1FFFFFu;
        out[5] = (uint32_t)(cs >> 43);
    }
    __device__ __forceinline__ void term(uint64_t a, const uint32_t *c)
    {
        const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
        A0 += (uint64_t)a0 * c[0];
        A1 += (uint64_t)a0 * c[1];
        A2 += (uint64_t)a0 * c[2];
        A0 += (uint64_t)a1 * c[3];
        A1 += (uint64_t)a1 * c[4];
        A2 += (uint64_t)a1 * c[5];
    }
    // the same from a 16-byte aligned limb slot (one 16-byte + one 8-byte load;
    // ZK_LIMB_AS: the address space a run-time compiled kernel reads its limb
    // table through, csrc/zxp_jit.hip)
    __device__ __forceinline__ void term_al(uint64_t a, const uint32_t *c)
    {
#if defined(ZK_LIMB_AS)
        typedef uint32_t u32x4_ __attribute__((ext_vector_type(4)));
        typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
        const u32x4_ qv = *(const ZK_LIMB_AS u32x4_ *)c;
        const u32x2_ rv = *(const ZK_LIMB_AS u32x2_ *)(c + 4);
        const LimbQ q{qv.x, qv.y, qv.z, qv.w};
        const LimbP r{rv.x, rv.y};
#elif defined(ZK_LIMB_STRUCT)
        // a whole-table LDS copy read by an -O2 kernel (zxp_jit.hip): the
        // load/store vectorizer merges the struct copy itself; explicit vector
        // loads there cost the config-4 quotient 13.3 -> 16.3 ms
        const LimbQ q = *(const LimbQ *)c;
        const LimbP r = *(const LimbP *)(c + 4);
#else
        // explicit vector types: a struct copy is split into dword loads at
        // -O1, which the LDS chunks of the split programs then read as
        // ds_read2_b32 pairs, each behind a v_add_u32 of its base (the pair's
        // 8-bit offsets do not reach across a 4 KB chunk); one 16-byte and one
        // 8-byte read take the 16-bit offset field instead
        typedef uint32_t u32x4_ __attribute__((ext_vector_type(4)));
        typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
        const u32x4_ qv = *(const u32x4_ *)c;
        const u32x2_ rv = *(const u32x2_ *)(c + 4);
        const LimbQ q{qv.x, qv.y, qv.z, qv.w};
        const LimbP r{rv.x, rv.y};
#endif
        const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
        A0 += (uint64_t)a0 * q.x;
        A1 += (uint64_t)a0 * q.y;
        A2 += (uint64_t)a0 * q.z;
        A0 += (uint64_t)a1 * q.w;
        A1 += (uint64_t)a1 * r.x;
        A2 += (uint64_t)a1 * r.y;
    }
    // coefficient 1: a0 -> A0, a1 * 2^32 = a1 * 2^10 * 2^22 -> A1
    __device__ __forceinline__ void lane(uint64_t a)
    {
        A0 += (uint32_t)a;
        A1 += (uint64_t)(uint32_t)(a >> 32) << 10;
    }
    __device__ __forceinline__ uint64_t fin() const
    {
        uint64_t l1, l2;
        const uint32_t c1 = __builtin_add_overflow(A0, A1 << 22, &l1) ? 1u : 0u;
        const uint32_t c2 = __builtin_add_overflow(l1, A2 << 43, &l2) ? 1u : 0u;
        const uint64_t h = (A1 >> 42) + (A2 >> 21) + c1 + c2;  // < 2^41
        return gl_reduce128(l2, h);
    }
};

}  // namespace zk
