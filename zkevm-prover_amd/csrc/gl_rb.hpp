// Goldilocks helpers whose final correction is rare: taken behind a
// wave-uniform branch (the compare's lane mask is the ballot, the branch is
// scalar), so the common path drops the select and the 64-bit add.  Same
// values as the gl_device.hpp forms, bit for bit.  Kept out of
// gl_device.hpp, whose text is part of every run-time compiled expression
// kernel's source (and code-object cache key).
#pragma once
#include "gl_device.hpp"

namespace zk {

// gl_reduce128 with the rare correction of lo - hh (a borrow needs lo < hh <
// 2^32: about 2^-32 of products)
__device__ __forceinline__ uint64_t gl_reduce128_rb(uint64_t lo, uint64_t hi)
{
    const uint32_t hh = (uint32_t)(hi >> 32);
    const uint32_t hl = (uint32_t)hi;
    uint64_t t0, r;
    const bool br = __builtin_sub_overflow(lo, (uint64_t)hh, &t0);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(br) != 0, 0)) t0 -= br ? ZK_EPS : 0ULL;
    const uint64_t t1 = ((uint64_t)hl << 32) - hl;
    const bool c = __builtin_add_overflow(t0, t1, &r);
    return r + (c ? ZK_EPS : 0ULL);
}

// lo + hl 2^64 for a small hl (< 2^20: hl EPS < 2^52, so the carry needs lo
// >= 2^64 - 2^52, about 2^-12; the Poseidon MDS row sums have hl < 2^11)
__device__ __forceinline__ uint64_t gl_reduce96_small_rb(uint64_t lo, uint32_t hl)
{
    const uint64_t t1 = ((uint64_t)hl << 32) - hl;
    uint64_t r;
    const bool c = __builtin_add_overflow(lo, t1, &r);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(c) != 0, 0)) r += c ? ZK_EPS : 0ULL;
    return r;
}

// Dot3::fin with the reduction's rare correction (the sum's high word is
// < 2^41, so lo - hh borrows with probability < 2^-55)
__device__ __forceinline__ uint64_t dot3_fin_rb(const Dot3 &d)
{
    uint64_t l1, l2;
    const uint32_t c1 = __builtin_add_overflow(d.A0, d.A1 << 22, &l1) ? 1u : 0u;
    const uint32_t c2 = __builtin_add_overflow(l1, d.A2 << 43, &l2) ? 1u : 0u;
    const uint64_t h = (d.A1 >> 42) + (d.A2 >> 21) + c1 + c2;
    return gl_reduce128_rb(l2, h);
}

__device__ __forceinline__ uint64_t gl_mul_rb(uint64_t a, uint64_t b)
{
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
    const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
    const uint64_t hi = (uint64_t)a1 * b1 + (t >> 32) + (u >> 32);
    const uint64_t lo = (u << 32) | (uint32_t)p00;
    return gl_reduce128_rb(lo, hi);
}

// mul2e with its final correction behind a wave-uniform branch where that
// correction is rare (the radix-256 NTT pass; same values as mul2e): for
// 0 < E < 32 the carry of lo + hl EPS needs lo >= 2^64 - 2^(E+32) (about
// 2^(E-32) per lane, so a 64-lane wave takes it with probability ~2^(E-26):
// the branch pays only for E <= ZK_RB_SHIFT_MAX_E), for 32 < E < 96 the
// borrow needs the shifted high word below 2^2 (about 2^-30).  E = 32,
// E >= 96 and the larger E < 32 keep mul2e.
#ifndef ZK_RB_SHIFT_MAX_E
#define ZK_RB_SHIFT_MAX_E 20
#endif
template <int E>
__device__ __forceinline__ uint64_t mul2e_rb(uint64_t x)
{
    static_assert(E >= 0 && E < 192, "exponent range");
    if constexpr (E == 0 || E == 32 || E >= 96 || (E < 32 && E > ZK_RB_SHIFT_MAX_E)) {
        return mul2e<E>(x);
    } else if constexpr (E < 32) {
        const uint32_t hl = (uint32_t)(x >> (64 - E));
        const uint64_t t1 = ((uint64_t)hl << 32) - hl;
        uint64_t r;
        const bool c = __builtin_add_overflow(x << E, t1, &r);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(c) != 0, 0)) r += c ? ZK_EPS : 0ULL;
        return r;
    } else if constexpr (E < 64) {
        constexpr int k = E - 32;
        const uint64_t lo = x << k;
        const uint32_t hl = (uint32_t)(x >> (64 - k));
        const uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32);
        uint32_t s1;
        const uint32_t s0 = __builtin_addc(l0, l1, 0u, &s1);
        const uint64_t u = ((uint64_t)s0 << 32) | (s1 ? 0xFFFFFFFFu : 0u);
        uint64_t r;
        const bool b = __builtin_sub_overflow(u, (uint64_t)l1 + hl, &r);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(b) != 0, 0)) r -= b ? ZK_EPS : 0ULL;
        return r;
    } else {
        constexpr int k = E - 64;
        const uint64_t lo = x << k;
        const uint32_t hl = k ? (uint32_t)(x >> (64 - (k ? k : 1))) : 0u;
        const uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32);
        const uint32_t a = l0 - hl;
        const uint64_t c = (uint64_t)l0 + l1 + (hl > l0 ? ZK_EPS : 0ULL);
        uint64_t r;
        const bool b = __builtin_sub_overflow((uint64_t)a << 32, c, &r);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(b) != 0, 0)) r -= b ? ZK_EPS : 0ULL;
        return r;
    }
}

}  // namespace zk
