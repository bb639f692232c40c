// Poseidon-GL permutation (t = 12, RF = 8, RP = 22, x^7) for gfx950 device code.
//
// Two exact evaluations of the reference's permutation
// (poseidon_g_executor.cpp:201-231; PoseidonGoldilocks::hash_full_result):
//
//  * perm_textbook: every round = add constants, S-box, 12x12 MDS.
//  * perm_sparse:   full rounds as above; the 22 partial rounds in the sparse
//    form of tools/gen_poseidon_sparse.py (one dense 11x11 matrix, then per
//    round 22 products instead of a 12x12 MDS).  Same output bit for bit.
//
// MDS (full rounds): the entries are < 64 and each row sums to < 2^9, so each
// lane is split into 22/22/20-bit limbs and every limb's dot product is
// accumulated with full-rate 24-bit multiply-adds (v_mad_u32_u24, MDS entries
// as inline constants) in 32 bits without overflow; one 96-bit recombination
// and a reduction per output lane.
#pragma once
#include "gl_device.hpp"
#include "gl_rb.hpp"
#include "poseidon_gl_constants.h"
#include "poseidon_gl_sparse.h"

#include <utility>

namespace zk {

#ifndef ZKGPU_POSEIDON_RB
#define ZKGPU_POSEIDON_RB 1
#endif

// a partial-round dot product's final reduction
__device__ __forceinline__ uint64_t pfin(const Dot3 &d) { return ZKGPU_POSEIDON_RB ? dot3_fin_rb(d) : d.fin(); }

// gl_mul specialised for squaring: 3 partial products instead of 4
__device__ __forceinline__ uint64_t gl_sqr3(uint64_t a)
{
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint64_t p00 = (uint64_t)a0 * a0;
    const uint64_t p01 = (uint64_t)a0 * a1;  // appears twice
    const uint64_t p11 = (uint64_t)a1 * a1;
    // a^2 = p00 + 2*p01*2^32 + p11*2^64
    const uint64_t t = p01 + (p00 >> 32);                 // < 2^64
    const uint64_t u = p01 + (uint32_t)t;                 // < 2^64
    const uint64_t hi = p11 + (t >> 32) + (u >> 32);
    const uint64_t lo = (u << 32) | (uint32_t)p00;
    return ZKGPU_POSEIDON_RB ? gl_reduce128_rb(lo, hi) : gl_reduce128(lo, hi);
}

// S-box products with the reduction's rare correction behind a uniform
// branch (gl_rb.hpp): 3 fewer VALU per product, 4 products per S-box
__device__ __forceinline__ uint64_t pow7(uint64_t x)
{
    const uint64_t x2 = gl_sqr3(x);
    const uint64_t x3 = ZKGPU_POSEIDON_RB ? gl_mul_rb(x2, x) : gl_mul(x2, x);
    const uint64_t x4 = gl_sqr3(x2);
    return ZKGPU_POSEIDON_RB ? gl_mul_rb(x3, x4) : gl_mul(x3, x4);
}

// M[x][y] = MCIRC[(y - x) mod 12] + (x == y == 0) * 8
__device__ __host__ constexpr uint32_t mds_entry(int x, int y)
{
    constexpr uint32_t MC[12] = {17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20};
    return MC[(y - x + 12) % 12] + ((x == 0 && y == 0) ? 8u : 0u);
}

// Reference form: 32-bit halves with 32x32->64 multiply-adds.
__device__ __forceinline__ void mds_halves(uint64_t st[12])
{
    uint32_t lo[12], hi[12];
#pragma unroll
    for (int y = 0; y < 12; y++) {
        lo[y] = (uint32_t)st[y];
        hi[y] = (uint32_t)(st[y] >> 32);
    }
    uint64_t out[12];
#pragma unroll
    for (int x = 0; x < 12; x++) {
        uint64_t sl = 0, sh = 0;
#pragma unroll
        for (int y = 0; y < 12; y++) {
            sl += (uint64_t)lo[y] * mds_entry(x, y);
            sh += (uint64_t)hi[y] * mds_entry(x, y);
        }
        uint64_t l = sl + (sh << 32);
        uint64_t c = (l < sl) ? 1ULL : 0ULL;
        uint64_t h = (sh >> 32) + c;
        out[x] = gl_reduce128(l, h);
    }
#pragma unroll
    for (int x = 0; x < 12; x++) st[x] = out[x];
}

// 22/22/20-bit limbs, 24-bit multiply-adds (full rate).
__device__ __forceinline__ void mds_limbs(uint64_t st[12])
{
    uint32_t a[12], b[12], c[12];
#pragma unroll
    for (int y = 0; y < 12; y++) {
        const uint32_t lo = (uint32_t)st[y], hi = (uint32_t)(st[y] >> 32);
        a[y] = lo & 0x3FFFFFu;
        b[y] = __builtin_amdgcn_alignbit(hi, lo, 22) & 0x3FFFFFu;
        c[y] = hi >> 12;
    }
    uint64_t out[12];
#pragma unroll
    for (int x = 0; x < 12; x++) {
        uint32_t A = 0, B = 0, C = 0;
#pragma unroll
        for (int y = 0; y < 12; y++) {
            A = __umul24(a[y], mds_entry(x, y)) + A;
            B = __umul24(b[y], mds_entry(x, y)) + B;
            C = __umul24(c[y], mds_entry(x, y)) + C;
        }
        // value = A + B*2^22 + C*2^44, A, B, C < 2^31
        const uint64_t t = (uint64_t)A + ((uint64_t)B << 22);  // < 2^54
        const uint64_t u = (uint64_t)C << 44;                   // low 64 bits of C*2^44
        uint64_t lo;
        const bool cy = __builtin_add_overflow(t, u, &lo);
        const uint32_t hi = (C >> 20) + (cy ? 1u : 0u);         // < 2^12
        out[x] = gl_reduce96(lo, hi);
    }
#pragma unroll
    for (int x = 0; x < 12; x++) st[x] = out[x];
}

template <bool LIMBS>
__device__ __forceinline__ void mds(uint64_t st[12])
{
    if constexpr (LIMBS)
        mds_limbs(st);
    else
        mds_halves(st);
}

// Sum of products of lazy elements, reduced once: each 128-bit product
// l + 2^64 h is added into lo (carries counted into the 2^64 place) and h
// into mid (carries counted into the 2^128 place == -2^32 mod p).
struct AccGL {
    uint64_t lo = 0, mid = 0;
    uint32_t c64 = 0, c128 = 0;
    __device__ __forceinline__ void mac(uint64_t a, uint64_t b)
    {
        const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
        const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
        const uint64_t p00 = (uint64_t)a0 * b0;
        const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
        const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
        const uint64_t h = (uint64_t)a1 * b1 + (t >> 32) + (u >> 32);
        const uint64_t l = (u << 32) | (uint32_t)p00;
        uint64_t s;
        c64 += __builtin_add_overflow(lo, l, &s) ? 1u : 0u;
        lo = s;
        c128 += __builtin_add_overflow(mid, h, &s) ? 1u : 0u;
        mid = s;
    }
    // add a lazy element (no product)
    __device__ __forceinline__ void add(uint64_t a)
    {
        uint64_t s;
        c64 += __builtin_add_overflow(lo, a, &s) ? 1u : 0u;
        lo = s;
    }
    __device__ __forceinline__ uint64_t reduce() const
    {
        uint64_t m;
        const uint32_t c2 = c128 + (__builtin_add_overflow(mid, (uint64_t)c64, &m) ? 1u : 0u);
        // lo + 2^64 m + 2^128 c2,  2^128 == -2^32 (mod p)
        return gl_sub(gl_reduce128(lo, m), (uint64_t)c2 << 32);
    }
};

// a + b*c  (mod p), lazy: one 128-bit product plus a 64-bit addend, one reduction
__device__ __forceinline__ uint64_t gl_madd(uint64_t a, uint64_t b, uint64_t c)
{
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint32_t c0 = (uint32_t)c, c1 = (uint32_t)(c >> 32);
    const uint64_t p00 = (uint64_t)b0 * c0;
    const uint64_t t = (uint64_t)b0 * c1 + (p00 >> 32);
    const uint64_t u = (uint64_t)b1 * c0 + (uint32_t)t;
    uint64_t h = (uint64_t)b1 * c1 + (t >> 32) + (u >> 32);  // <= 2^64 - 2
    const uint64_t l = (u << 32) | (uint32_t)p00;
    uint64_t s;
    h += __builtin_add_overflow(l, a, &s) ? 1ULL : 0ULL;
    return gl_reduce128(s, h);
}

template <bool LIMBS>
__device__ __forceinline__ void full_round(uint64_t st[12], int r)
{
#pragma unroll
    for (int s = 0; s < 12; s++) st[s] = pow7(gl_add(st[s], ZKGPU_POSEIDON_RC[r * 12 + s]));
    mds<LIMBS>(st);
}

// textbook permutation (reference form)
template <bool LIMBS>
__device__ __forceinline__ void perm_textbook(uint64_t st[12])
{
#pragma unroll 1
    for (int r = 0; r < 4; r++) full_round<LIMBS>(st, r);
#pragma unroll 1
    for (int r = 4; r < 26; r++) {
#pragma unroll
        for (int s = 0; s < 12; s++) st[s] = gl_add(st[s], ZKGPU_POSEIDON_RC[r * 12 + s]);
        st[0] = pow7(st[0]);
        mds<LIMBS>(st);
    }
#pragma unroll 1
    for (int r = 26; r < 30; r++) full_round<LIMBS>(st, r);
}

// sparse partial rounds (tools/gen_poseidon_sparse.py), bit-identical output
template <bool LIMBS>
__device__ __forceinline__ void perm_sparse(uint64_t st[12])
{
#pragma unroll 1
    for (int r = 0; r < 4; r++) full_round<LIMBS>(st, r);
    {
        uint64_t in[11];
#pragma unroll
        for (int j = 0; j < 11; j++) in[j] = gl_add(st[1 + j], ZKGPU_PSP_PRE[1 + j]);
        st[0] = gl_add(st[0], ZKGPU_PSP_PRE[0]);
#pragma unroll
        for (int i = 0; i < 11; i++) {
            AccGL acc;
#pragma unroll
            for (int j = 0; j < 11; j++) acc.mac(in[j], ZKGPU_PSP_D0[i * 11 + j]);
            st[1 + i] = acc.reduce();
        }
    }
#pragma unroll 1
    for (int k = 0; k < 22; k++) {
        const uint64_t s0 = gl_add(pow7(st[0]), ZKGPU_PSP_POST[k]);
        AccGL acc;
        // 25 * s0 < 2^69: as a product with a small constant
        acc.mac(s0, 25);
#pragma unroll
        for (int j = 0; j < 11; j++) acc.mac(st[1 + j], ZKGPU_PSP_W[k * 11 + j]);
#pragma unroll
        for (int j = 0; j < 11; j++) st[1 + j] = gl_madd(st[1 + j], s0, ZKGPU_PSP_V[k * 11 + j]);
        st[0] = acc.reduce();
    }
#pragma unroll 1
    for (int r = 26; r < 30; r++) full_round<LIMBS>(st, r);
}

// ------------------------------------------------------------------ fast form
// MDS on 32-bit halves with a constant vector K folded into the accumulators:
// st = M * st + K.  (K = the next round's constants, so no separate add.)
// The matrix entries go through an empty asm so the compiler keeps plain
// 32x32+64 multiply-adds: its shift-add strength reduction for the entries 2,
// 8 and 16 needs zero-extended 64-bit operands (one move each).  The 75-bit
// row sum is recombined with a 32-bit carry chain.  538 -> 438 VALU per MDS.
__device__ __forceinline__ void mds_fold(uint64_t st[12], const uint64_t *K)
{
    uint32_t lo[12], hi[12];
#pragma unroll
    for (int y = 0; y < 12; y++) {
        lo[y] = (uint32_t)st[y];
        hi[y] = (uint32_t)(st[y] >> 32);
    }
    uint32_t c[13];
#pragma unroll
    for (int j = 0; j < 12; j++) {
        c[j] = mds_entry(0, j) - (j == 0 ? 8u : 0u);  // MCIRC[j]
        asm volatile("" : "+s"(c[j]));
    }
    c[12] = 8;  // MDIAG[0]
    asm volatile("" : "+s"(c[12]));
#pragma unroll
    for (int x = 0; x < 12; x++) {
        uint64_t sl = (uint32_t)K[x], sh = K[x] >> 32;
#pragma unroll
        for (int y = 0; y < 12; y++) {
            const uint32_t e = c[(y - x + 12) % 12];
            sl += (uint64_t)lo[y] * e;
            sh += (uint64_t)hi[y] * e;
        }
        if (x == 0) {
            sl += (uint64_t)lo[0] * c[12];
            sh += (uint64_t)hi[0] * c[12];
        }
        // value = sl + sh * 2^32 < 2^75: (h : mid : sl0)
        uint32_t c1, c2;
        const uint32_t mid = __builtin_addc((uint32_t)(sl >> 32), (uint32_t)sh, 0u, &c1);
        const uint32_t h = __builtin_addc((uint32_t)(sh >> 32), 0u, c1, &c2);
        st[x] = ZKGPU_POSEIDON_RB ? gl_reduce96_small_rb(((uint64_t)mid << 32) | (uint32_t)sl, h)
                                  : gl_reduce96(((uint64_t)mid << 32) | (uint32_t)sl, h);
    }
}

// Circulant part of the MDS on 32-bit halves, in the frequency domain
// (tools/mds_fft.py checks the algebra): Good-Thomas maps the length-12 cyclic
// convolution y = r * v (r_k = MCIRC[-k]) onto 4 x 3, n = (9a + 4b) mod 12.
// Along a, X^4 - 1 = (X - 1)(X + 1)(X^2 + 1); along b, 3-point cyclic
// convolutions with the transformed kernel, which for this matrix is all
// signed powers of two once the inverse's 1/4 and 1/2 are folded in:
//   (X - 1): [16, 32, 16]   (X + 1): [-1, 8, 2]   (X^2 + 1): [2 - i, -1 - 4i, -16 - i]
// so every product is a shift.  Wrapping u64 arithmetic is exact: the
// outputs are the (non-negative, < 2^41) integer row sums.
__device__ __forceinline__ void mds_circ_fft(const uint64_t v[12], uint64_t w[12])
{
    uint64_t u0[3], u1[3], p[3], q[3];
#pragma unroll
    for (int b = 0; b < 3; b++) {
        const uint64_t S0 = v[(4 * b) % 12], S1 = v[(9 + 4 * b) % 12], S2 = v[(18 + 4 * b) % 12],
                       S3 = v[(27 + 4 * b) % 12];
        const uint64_t t0 = S0 + S2, t1 = S1 + S3;
        u0[b] = t0 + t1;
        u1[b] = t0 - t1;
        p[b] = S0 - S2;
        q[b] = S1 - S3;
    }
    const uint64_t s0 = u0[0] + u0[1] + u0[2];
#pragma unroll
    for (int b = 0; b < 3; b++) {
        const int b1 = (b + 2) % 3, b2 = (b + 1) % 3;  // b - 1, b - 2
        const uint64_t V0 = (s0 + u0[b1]) << 4;
        const uint64_t V1 = (u1[b1] << 3) + (u1[b2] << 1) - u1[b];
        const uint64_t re = (p[b] << 1) + q[b] + (q[b1] << 2) + q[b2] - p[b1] - (p[b2] << 4);
        const uint64_t im = (q[b] << 1) - p[b] - q[b1] - (p[b1] << 2) - (q[b2] << 4) - p[b2];
        const uint64_t A = V0 + V1, B = V0 - V1;
        w[(4 * b) % 12] = A + re;
        w[(18 + 4 * b) % 12] = A - re;
        w[(9 + 4 * b) % 12] = B + im;
        w[(27 + 4 * b) % 12] = B - im;
    }
}

// st = M * st + K with the circulant part from mds_circ_fft (same result as
// mds_fold, bit for bit)
__device__ __forceinline__ void mds_fft_fold(uint64_t st[12], const uint64_t *K)
{
    uint64_t lo[12], hi[12], wl[12], wh[12];
#pragma unroll
    for (int y = 0; y < 12; y++) {
        lo[y] = (uint32_t)st[y];
        hi[y] = st[y] >> 32;
    }
    mds_circ_fft(lo, wl);
    mds_circ_fft(hi, wh);
    wl[0] += lo[0] << 3;  // MDIAG[0] = 8
    wh[0] += hi[0] << 3;
#pragma unroll
    for (int x = 0; x < 12; x++) {
        const uint64_t sl = wl[x] + (uint32_t)K[x], sh = wh[x] + (K[x] >> 32);
        // value = sl + sh * 2^32 < 2^75: (h : mid : sl0)
        uint32_t c1, c2;
        const uint32_t mid = __builtin_addc((uint32_t)(sl >> 32), (uint32_t)sh, 0u, &c1);
        const uint32_t h = __builtin_addc((uint32_t)(sh >> 32), 0u, c1, &c2);
        st[x] = ZKGPU_POSEIDON_RB ? gl_reduce96_small_rb(((uint64_t)mid << 32) | (uint32_t)sl, h)
                                  : gl_reduce96(((uint64_t)mid << 32) | (uint32_t)sl, h);
    }
}

#ifndef ZKGPU_MDS_FFT
#define ZKGPU_MDS_FFT 1
#endif

// Dot3 (table-coefficient dot products): csrc/gl_device.hpp

static constexpr uint64_t ZKGPU_PS_ZERO12[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

__device__ __forceinline__ void full_rounds_fold(uint64_t st[12], int r0)
{
#pragma unroll 1
    for (int r = r0; r < r0 + 4; r++) {
#pragma unroll
        for (int s = 0; s < 12; s++) st[s] = pow7(st[s]);
        const uint64_t *K = r == 3 ? ZKGPU_PSP_PRE : (r == 29 ? ZKGPU_PS_ZERO12 : &ZKGPU_POSEIDON_RC[(r + 1) * 12]);
        if constexpr (ZKGPU_MDS_FFT)
            mds_fft_fold(st, K);
        else
            mds_fold(st, K);
    }
}

// table offset of the x-dot of block step t (3 + 6 + 66 + 6t words each)
__host__ __device__ constexpr int psb_xoff(int t) { return 75 * t + 3 * t * (t - 1); }

template <int t>
__device__ __forceinline__ void psb_step(uint64_t &x, uint64_t y[], const uint64_t L[11], const uint32_t *T)
{
    constexpr int o = psb_xoff(t);
    y[t] = pow7(x);
    Dot3 d(T + o);
    d.term(y[t], T + o + 3);
#pragma unroll
    for (int j = 0; j < 11; j++) d.term(L[j], T + o + 9 + 6 * j);
#pragma unroll
    for (int i = 0; i < t; i++) d.term(y[i], T + o + 75 + 6 * i);
    x = pfin(d);
}

template <int... ts>
__device__ __forceinline__ void psb_steps(uint64_t &x, uint64_t y[], const uint64_t L[11], const uint32_t *T,
                                          std::integer_sequence<int, ts...>)
{
    (psb_step<ts>(x, y, L, T), ...);
}

// Partial rounds in block dot-product form (gen_poseidon_sparse.py
// derive_blocks); input: lanes after the first four full rounds (PRE added),
// output: lanes with the round-26 constants added.  D0 / BL: the tables
// ZKGPU_PSB_D0 / ZKGPU_PSB_BLOCKS (compile-time by default; a copy in
// memory the compiler cannot fold is read with scalar loads instead of one
// s_mov per coefficient)
template <typename TP = const uint32_t *>
__device__ __forceinline__ void partial_rounds_blocks(uint64_t st[12], TP D0 = ZKGPU_PSB_D0, TP BL = ZKGPU_PSB_BLOCKS)
{
    uint64_t L[11];
#pragma unroll
    for (int i = 0; i < 11; i++) {
        Dot3 d(&D0[i * 69]);
#pragma unroll
        for (int j = 0; j < 11; j++) d.term(st[1 + j], &D0[i * 69 + 3 + 6 * j]);
        L[i] = pfin(d);
    }
    uint64_t x = st[0];
#pragma unroll 1
    for (int b = 0; b < ZKGPU_PSB_NBLOCKS; b++) {
        const uint32_t *T = &BL[b * ZKGPU_PSB_BLOCK_WORDS];
        uint64_t y[ZKGPU_PSB_BLOCK];
        psb_steps(x, y, L, T, std::make_integer_sequence<int, ZKGPU_PSB_BLOCK>{});
        constexpr int base = psb_xoff(ZKGPU_PSB_BLOCK);
#pragma unroll
        for (int j = 0; j < 11; j++) {
            const uint32_t *Tj = T + base + j * (3 + 6 * ZKGPU_PSB_BLOCK);
            Dot3 d(Tj);
            d.lane(L[j]);
#pragma unroll
            for (int i = 0; i < ZKGPU_PSB_BLOCK; i++) d.term(y[i], Tj + 3 + 6 * i);
            L[j] = pfin(d);
        }
    }
    st[0] = x;
#pragma unroll
    for (int j = 0; j < 11; j++) st[1 + j] = L[j];
}

__device__ __forceinline__ void perm_fast(uint64_t st[12])
{
#pragma unroll
    for (int s = 0; s < 12; s++) st[s] = gl_add(st[s], ZKGPU_POSEIDON_RC[s]);
    full_rounds_fold(st, 0);
    partial_rounds_blocks(st);
    full_rounds_fold(st, 26);
}

// perm_fast with the partial-round tables read from memory (D0, BL: copies
// of ZKGPU_PSB_D0 / ZKGPU_PSB_BLOCKS); bit-identical
__device__ __forceinline__ void perm_fast_tab(uint64_t st[12], const uint32_t *D0, const uint32_t *BL)
{
#pragma unroll
    for (int s = 0; s < 12; s++) st[s] = gl_add(st[s], ZKGPU_POSEIDON_RC[s]);
    full_rounds_fold(st, 0);
    partial_rounds_blocks(st, D0, BL);
    full_rounds_fold(st, 26);
}

// ---- K independent permutations per thread, step by step interleaved: the
// partial rounds are one serial chain per state (S-box of s0 -> dot product
// -> next S-box), so a second state doubles the independent work the
// scheduler has to hide that chain's latency
template <int K>
__device__ __forceinline__ void full_rounds_fold_k(uint64_t (*st)[12], int r0)
{
#pragma unroll 1
    for (int r = r0; r < r0 + 4; r++) {
#pragma unroll
        for (int k = 0; k < K; k++)
#pragma unroll
            for (int s = 0; s < 12; s++) st[k][s] = pow7(st[k][s]);
        const uint64_t *Kc = r == 3 ? ZKGPU_PSP_PRE : (r == 29 ? ZKGPU_PS_ZERO12 : &ZKGPU_POSEIDON_RC[(r + 1) * 12]);
#pragma unroll
        for (int k = 0; k < K; k++) {
            if constexpr (ZKGPU_MDS_FFT)
                mds_fft_fold(st[k], Kc);
            else
                mds_fold(st[k], Kc);
        }
    }
}

// SPLIT: each dot product in two halves summed at the end (two independent
// multiply-add chains per accumulator instead of one; the sum of the halves'
// carry-free accumulators is the same integer)
template <int K, bool SPLIT, int t>
__device__ __forceinline__ void psb_step_k(uint64_t *x, uint64_t (*y)[ZKGPU_PSB_BLOCK], const uint64_t (*L)[11],
                                           const uint32_t *T)
{
    constexpr int o = psb_xoff(t);
#pragma unroll
    for (int k = 0; k < K; k++) y[k][t] = pow7(x[k]);
#pragma unroll
    for (int k = 0; k < K; k++) {
        Dot3 d(T + o);
        if constexpr (SPLIT) {
            Dot3 e;
            d.term(y[k][t], T + o + 3);
#pragma unroll
            for (int j = 0; j < 11; j++) {
                if (j & 1) d.term(L[k][j], T + o + 9 + 6 * j);
                else e.term(L[k][j], T + o + 9 + 6 * j);
            }
#pragma unroll
            for (int i = 0; i < t; i++) {
                if (i & 1) e.term(y[k][i], T + o + 75 + 6 * i);
                else d.term(y[k][i], T + o + 75 + 6 * i);
            }
            d.A0 += e.A0;
            d.A1 += e.A1;
            d.A2 += e.A2;
        } else {
            d.term(y[k][t], T + o + 3);
#pragma unroll
            for (int j = 0; j < 11; j++) d.term(L[k][j], T + o + 9 + 6 * j);
#pragma unroll
            for (int i = 0; i < t; i++) d.term(y[k][i], T + o + 75 + 6 * i);
        }
        x[k] = pfin(d);
    }
}

template <int K, bool SPLIT, int... ts>
__device__ __forceinline__ void psb_steps_k(uint64_t *x, uint64_t (*y)[ZKGPU_PSB_BLOCK], const uint64_t (*L)[11],
                                            const uint32_t *T, std::integer_sequence<int, ts...>)
{
    (psb_step_k<K, SPLIT, ts>(x, y, L, T), ...);
}

template <int K, bool SPLIT>
__device__ __forceinline__ void partial_rounds_blocks_k(uint64_t (*st)[12])
{
    uint64_t L[K][11];
#pragma unroll
    for (int k = 0; k < K; k++)
#pragma unroll
        for (int i = 0; i < 11; i++) {
            Dot3 d(&ZKGPU_PSB_D0[i * 69]);
#pragma unroll
            for (int j = 0; j < 11; j++) d.term(st[k][1 + j], &ZKGPU_PSB_D0[i * 69 + 3 + 6 * j]);
            L[k][i] = pfin(d);
        }
    uint64_t x[K];
#pragma unroll
    for (int k = 0; k < K; k++) x[k] = st[k][0];
#pragma unroll 1
    for (int b = 0; b < ZKGPU_PSB_NBLOCKS; b++) {
        const uint32_t *T = &ZKGPU_PSB_BLOCKS[b * ZKGPU_PSB_BLOCK_WORDS];
        uint64_t y[K][ZKGPU_PSB_BLOCK];
        psb_steps_k<K, SPLIT>(x, y, L, T, std::make_integer_sequence<int, ZKGPU_PSB_BLOCK>{});
        constexpr int base = psb_xoff(ZKGPU_PSB_BLOCK);
#pragma unroll
        for (int k = 0; k < K; k++)
#pragma unroll
            for (int j = 0; j < 11; j++) {
                const uint32_t *Tj = T + base + j * (3 + 6 * ZKGPU_PSB_BLOCK);
                Dot3 d(Tj);
                d.lane(L[k][j]);
#pragma unroll
                for (int i = 0; i < ZKGPU_PSB_BLOCK; i++) d.term(y[k][i], Tj + 3 + 6 * i);
                L[k][j] = pfin(d);
            }
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        st[k][0] = x[k];
#pragma unroll
        for (int j = 0; j < 11; j++) st[k][1 + j] = L[k][j];
    }
}

// K permutations, bit-identical to K calls of perm_fast
template <int K, bool SPLIT = false>
__device__ __forceinline__ void perm_fast_k(uint64_t (*st)[12])
{
#pragma unroll
    for (int k = 0; k < K; k++)
#pragma unroll
        for (int s = 0; s < 12; s++) st[k][s] = gl_add(st[k][s], ZKGPU_POSEIDON_RC[s]);
    full_rounds_fold_k<K>(st, 0);
    partial_rounds_blocks_k<K, SPLIT>(st);
    full_rounds_fold_k<K>(st, 26);
}

// the permutation the product kernels use
__device__ __forceinline__ void poseidon_perm(uint64_t st[12]) { perm_fast(st); }

}  // namespace zk
