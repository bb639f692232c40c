// cpuref -- the CPU baseline of bench.py (cpu_baseline.kind
// "restated-reference-AVX2"): the reference's default CPU path for the
// proof's bulk kernels, restated -- NOT the checker (that is oracle/, which
// stays as it is) and never part of the product.
//
// The reference builds the Goldilocks library with AVX2 (Makefile:19) and
// hashes its Merkle trees with PoseidonGoldilocks::merkletree_avx
// (merkleTreeGL.cpp:37-44): OpenMP over rows, AVX2 field arithmetic, the
// permutation with the "optimised" sparse partial rounds (Poseidon paper,
// appendix B; the goldilocks submodule is absent, its algorithm is
// restated).  Its NTT is the blocked row-major radix-2 of
// tools/starkpil/bctree/build_const_tree.cpp:216-533 (whole rows of columns
// per butterfly, the first stages inside cache blocks), vectorised over the
// columns.  Here:
//   * 4-lane AVX2 Goldilocks arithmetic (64x64 products from four
//     _mm256_mul_epu32, the 2^64 = 2^32 - 1 fold, lazy values < 2^64);
//   * the permutation on 4 states at once (one per 64-bit lane): 4 + 4 full
//     rounds with the MDS as small-coefficient sums of 32-bit halves, the 22
//     partial rounds in the sparse form of zkevm-prover_amd/csrc/
//     poseidon_gl_sparse.h (the same constants the GPU uses: PRE, the 11x11
//     initial matrix, per round a lane-0 S-box, POST, the W / V vectors);
//   * linear_hash leaves of 4 rows per vector step, tree levels 4 nodes per
//     step, OpenMP over both;
//   * NTT / INTT / extendPol on row-major buffers, the oracle's blocked
//     schedule with the column loop vectorised.
// Bit-identical to the oracle (tests/test_cpuref.py).
#include <immintrin.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../zkevm-prover_amd/csrc/poseidon_gl_constants.h"
#include "../zkevm-prover_amd/csrc/poseidon_gl_sparse.h"

namespace {

typedef __m256i V;
constexpr uint64_t P = 0xFFFFFFFF00000001ULL;
constexpr uint64_t EPS = 0xFFFFFFFFULL;

// ---------------------------------------------------------------- scalar
inline uint64_t s_canon(uint64_t a) { return a >= P ? a - P : a; }
inline uint64_t s_reduce(unsigned __int128 x)
{
    const uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
    const uint64_t hh = hi >> 32, hl = hi & EPS;
    uint64_t t = lo - hh;
    if (lo < hh) t -= EPS;
    const uint64_t u = (hl << 32) - hl;
    uint64_t r = t + u;
    if (r < u) r += EPS;
    return r;
}
inline uint64_t s_mul(uint64_t a, uint64_t b) { return s_reduce((unsigned __int128)a * b); }
inline uint64_t s_add(uint64_t a, uint64_t b)  // b < p
{
    uint64_t s = a + b;
    if (s < a) s += EPS;
    return s;
}
inline uint64_t s_sub(uint64_t a, uint64_t b)  // b < p
{
    uint64_t d = a - b;
    if (a < b) d -= EPS;
    return d;
}
uint64_t s_pow(uint64_t a, uint64_t e)
{
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = s_mul(r, a);
        a = s_mul(a, a);
        e >>= 1;
    }
    return s_canon(r);
}
uint64_t s_w(unsigned n)  // Goldilocks::w(n)
{
    uint64_t w = 7277203076849721926ULL;
    for (unsigned i = n; i < 32; i++) w = s_mul(w, w);
    return s_canon(w);
}

// ---------------------------------------------------------------- AVX2
inline V bc(uint64_t x) { return _mm256_set1_epi64x((long long)x); }
inline V ltu(V a, V b)  // a < b, unsigned
{
    const V s = bc(1ULL << 63);
    return _mm256_cmpgt_epi64(_mm256_xor_si256(b, s), _mm256_xor_si256(a, s));
}
inline V v_canon(V a) { return _mm256_sub_epi64(a, _mm256_andnot_si256(ltu(a, bc(P)), bc(P))); }
inline V v_add(V a, V b)  // b < p; lazy result
{
    const V s = _mm256_add_epi64(a, b);
    return _mm256_add_epi64(s, _mm256_and_si256(ltu(s, a), bc(EPS)));
}
inline V v_sub(V a, V b)  // b < p
{
    const V d = _mm256_sub_epi64(a, b);
    return _mm256_sub_epi64(d, _mm256_and_si256(ltu(a, b), bc(EPS)));
}
// (hi, lo) -> lo - hi_hi + hi_lo (2^32 - 1) mod p, lazy
inline V v_reduce(V hi, V lo)
{
    const V hh = _mm256_srli_epi64(hi, 32), hl = _mm256_and_si256(hi, bc(EPS));
    V t = _mm256_sub_epi64(lo, hh);
    t = _mm256_sub_epi64(t, _mm256_and_si256(ltu(lo, hh), bc(EPS)));
    const V u = _mm256_sub_epi64(_mm256_slli_epi64(hl, 32), hl);
    const V r = _mm256_add_epi64(t, u);
    return _mm256_add_epi64(r, _mm256_and_si256(ltu(r, u), bc(EPS)));
}
inline V v_mul(V a, V b)
{
    const V ah = _mm256_srli_epi64(a, 32), bh = _mm256_srli_epi64(b, 32);
    const V ll = _mm256_mul_epu32(a, b), lh = _mm256_mul_epu32(a, bh), hl = _mm256_mul_epu32(ah, b),
            hh = _mm256_mul_epu32(ah, bh);
    const V t0 = _mm256_add_epi64(hl, _mm256_srli_epi64(ll, 32));  // < 2^64
    const V t1 = _mm256_add_epi64(lh, _mm256_and_si256(t0, bc(EPS)));
    const V hi = _mm256_add_epi64(_mm256_add_epi64(hh, _mm256_srli_epi64(t0, 32)), _mm256_srli_epi64(t1, 32));
    const V lo = _mm256_or_si256(_mm256_and_si256(ll, bc(EPS)), _mm256_slli_epi64(t1, 32));
    return v_reduce(hi, lo);
}
inline V v_pow7(V x)
{
    const V x2 = v_mul(x, x), x3 = v_mul(x2, x), x4 = v_mul(x2, x2);
    return v_mul(x3, x4);
}

// ---------------------------------------------------------------- Poseidon x4
const uint32_t MC[12] = {17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20};

// full round r: constants, S-box on every lane, MDS M[i][j] = MC[(j - i) mod
// 12] + (i == j == 0) * 8 as sums of coefficient x 32-bit half (< 2^42 each)
inline void full_round(V st[12], int r)
{
    V lo32[12], hi32[12];
    for (int i = 0; i < 12; i++) {
        const V x = v_canon(v_pow7(v_add(st[i], bc(ZKGPU_POSEIDON_RC[r * 12 + i]))));
        lo32[i] = x;  // (_mm256_mul_epu32 reads the low halves)
        hi32[i] = _mm256_srli_epi64(x, 32);
    }
    for (int i = 0; i < 12; i++) {
        V sl = _mm256_setzero_si256(), sh = _mm256_setzero_si256();
        for (int j = 0; j < 12; j++) {
            const V c = bc(MC[j >= i ? j - i : j + 12 - i] + (i == 0 && j == 0 ? 8 : 0));
            sl = _mm256_add_epi64(sl, _mm256_mul_epu32(lo32[j], c));
            sh = _mm256_add_epi64(sh, _mm256_mul_epu32(hi32[j], c));
        }
        // value = sl + sh 2^32 (< 2^75): lo = sl + (sh << 32), hi = sh >> 32 + carry
        const V shl = _mm256_slli_epi64(sh, 32);
        const V lo = _mm256_add_epi64(sl, shl);
        const V hi = _mm256_sub_epi64(_mm256_srli_epi64(sh, 32), ltu(lo, shl));  // (ltu mask = -1 on carry)
        st[i] = v_reduce(hi, lo);
    }
}

void perm4(V st[12])
{
    for (int r = 0; r < 4; r++) full_round(st, r);
    {
        V v[11];
        for (int j = 0; j < 11; j++) v[j] = v_canon(v_add(st[1 + j], bc(ZKGPU_PSP_PRE[1 + j])));
        st[0] = v_add(st[0], bc(ZKGPU_PSP_PRE[0]));
        for (int i = 0; i < 11; i++) {
            V acc = _mm256_setzero_si256();
            for (int j = 0; j < 11; j++) acc = v_add(acc, v_canon(v_mul(v[j], bc(ZKGPU_PSP_D0[i * 11 + j]))));
            st[1 + i] = acc;
        }
    }
    for (int k = 0; k < 22; k++) {
        const V s0 = v_canon(v_add(v_pow7(st[0]), bc(ZKGPU_PSP_POST[k])));
        V acc = v_canon(v_mul(s0, bc(25)));
        for (int j = 0; j < 11; j++) acc = v_add(acc, v_canon(v_mul(st[1 + j], bc(ZKGPU_PSP_W[k * 11 + j]))));
        for (int j = 0; j < 11; j++) st[1 + j] = v_add(st[1 + j], v_canon(v_mul(s0, bc(ZKGPU_PSP_V[k * 11 + j]))));
        st[0] = acc;
    }
    for (int r = 26; r < 30; r++) full_round(st, r);
}

// linear_hash of rows r0..r0+3 (row-major, ncols) into digests (4 each);
// nrow_valid < 4 repeats the last valid row (results discarded)
void leaves4(uint64_t *digests, const uint64_t *src, uint64_t ncols, uint64_t r0, uint64_t nvalid)
{
    alignas(32) uint64_t lane[4][12];
    const uint64_t *row[4];
    for (int l = 0; l < 4; l++) row[l] = src + (r0 + ((uint64_t)l < nvalid ? l : nvalid - 1)) * ncols;
    if (ncols <= 4) {
        for (uint64_t l = 0; l < nvalid; l++)
            for (int k = 0; k < 4; k++) digests[4 * (r0 + l) + k] = (uint64_t)k < ncols ? row[l][k] : 0;
        return;
    }
    V st[12];
    for (int k = 0; k < 12; k++) st[k] = _mm256_setzero_si256();
    for (uint64_t c0 = 0; c0 < ncols; c0 += 8) {
        const uint64_t nk = ncols - c0 < 8 ? ncols - c0 : 8;
        if (c0)
            for (int k = 0; k < 4; k++) st[8 + k] = st[k];
        for (int k = 0; k < 8; k++) {
            if ((uint64_t)k < nk)
                st[k] = v_canon(_mm256_set_epi64x((long long)row[3][c0 + k], (long long)row[2][c0 + k],
                                                  (long long)row[1][c0 + k], (long long)row[0][c0 + k]));
            else
                st[k] = _mm256_setzero_si256();
        }
        for (int k = 8; k < 12; k++) st[k] = v_canon(st[k]);
        perm4(st);
    }
    for (int k = 0; k < 4; k++) _mm256_store_si256((V *)lane[k], v_canon(st[k]));
    for (uint64_t l = 0; l < nvalid; l++)
        for (int k = 0; k < 4; k++) digests[4 * (r0 + l) + k] = lane[k][l];
}

// 4 parent nodes = hash(left || right) (capacity 0) of child pairs p0..p0+3
void nodes4(uint64_t *dst, const uint64_t *lvl, uint64_t p0, uint64_t nvalid)
{
    alignas(32) uint64_t lane[4][4];
    V st[12];
    for (int k = 0; k < 8; k++) {
        uint64_t x[4];
        for (int l = 0; l < 4; l++) x[l] = lvl[8 * (p0 + ((uint64_t)l < nvalid ? l : 0)) + k];
        st[k] = v_canon(_mm256_set_epi64x((long long)x[3], (long long)x[2], (long long)x[1], (long long)x[0]));
    }
    for (int k = 8; k < 12; k++) st[k] = _mm256_setzero_si256();
    perm4(st);
    for (int k = 0; k < 4; k++) _mm256_store_si256((V *)lane[k], v_canon(st[k]));
    for (uint64_t l = 0; l < nvalid; l++)
        for (int k = 0; k < 4; k++) dst[4 * (p0 + l) + k] = lane[k][l];
}

unsigned log2u(uint64_t n)
{
    unsigned l = 0;
    while ((1ULL << l) < n) l++;
    return l;
}
uint64_t bitrev(uint64_t x, unsigned bits)
{
    uint64_t r = 0;
    for (unsigned i = 0; i < bits; i++) {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

// butterfly of two rows (ncols values each) with twiddle w
inline void bfly(uint64_t *u, uint64_t *v, uint64_t w, uint64_t ncols)
{
    const V wv = bc(w);
    uint64_t c = 0;
    for (; c + 4 <= ncols; c += 4) {
        const V a = _mm256_loadu_si256((const V *)(u + c)), b = _mm256_loadu_si256((const V *)(v + c));
        const V t = v_canon(v_mul(b, wv));
        _mm256_storeu_si256((V *)(u + c), v_add(a, t));
        _mm256_storeu_si256((V *)(v + c), v_sub(a, t));
    }
    for (; c < ncols; c++) {
        const uint64_t t = s_canon(s_mul(v[c], w)), a = u[c];
        u[c] = s_add(a, t);
        v[c] = s_sub(a, t);
    }
}

constexpr unsigned BLOCK_BITS = 12;

// radix-2 DIT on bit-reversed rows: the first BLOCK_BITS stages inside
// blocks of 2^BLOCK_BITS rows (build_const_tree.cpp _fft_block), then the
// remaining stages across the blocks
void dit(uint64_t *x, uint64_t n, uint64_t ncols, uint64_t root)
{
    const unsigned L = log2u(n);
    if (!L) return;
    const uint64_t half_n = n >> 1;
    uint64_t *tw = (uint64_t *)malloc(8 * half_n);
#pragma omp parallel for schedule(static)
    for (uint64_t c = 0; c < half_n; c += 4096) {
        uint64_t v = s_pow(root, c);
        for (uint64_t k = c; k < c + 4096 && k < half_n; k++) {
            tw[k] = v;
            v = s_canon(s_mul(v, root));
        }
    }
    const unsigned B = L < BLOCK_BITS ? L : BLOCK_BITS;
    const uint64_t bsz = 1ULL << B;
#pragma omp parallel for schedule(static)
    for (uint64_t blk = 0; blk < n; blk += bsz)
        for (unsigned s = 1; s <= B; s++) {
            const uint64_t half = 1ULL << (s - 1), span = half << 1, ts = n >> s;
            for (uint64_t b = blk; b < blk + bsz; b += span)
                for (uint64_t i = 0; i < half; i++) bfly(x + (b + i) * ncols, x + (b + i + half) * ncols, tw[i * ts], ncols);
        }
    for (unsigned s = B + 1; s <= L; s++) {
        const uint64_t half = 1ULL << (s - 1), ts = n >> s;
#pragma omp parallel for schedule(static)
        for (uint64_t k = 0; k < half_n; k++) {
            const uint64_t i = k & (half - 1), b = (k >> (s - 1)) << s;
            bfly(x + (b + i) * ncols, x + (b + i + half) * ncols, tw[i * ts], ncols);
        }
    }
    free(tw);
}

void bitrev_rows(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols)
{
    const unsigned L = log2u(n);
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t *s = src + bitrev(i, L) * ncols;
        uint64_t *d = dst + i * ncols;
        for (uint64_t c = 0; c < ncols; c++) d[c] = s_canon(s[c]);
    }
}

// rows scaled by f0 * step^i, canonical
void scale_rows(uint64_t *x, uint64_t n, uint64_t ncols, uint64_t f0, uint64_t step)
{
#pragma omp parallel
    {
        const int T = omp_get_num_threads(), t = omp_get_thread_num();
        const uint64_t per = (n + T - 1) / T, a = per * t, e = a + per < n ? a + per : n;
        uint64_t f = s_canon(s_mul(f0, s_pow(step, a)));
        for (uint64_t i = a; i < e; i++) {
            uint64_t *r = x + i * ncols;
            const V fv = bc(f);
            uint64_t c = 0;
            for (; c + 4 <= ncols; c += 4)
                _mm256_storeu_si256((V *)(r + c), v_canon(v_mul(_mm256_loadu_si256((const V *)(r + c)), fv)));
            for (; c < ncols; c++) r[c] = s_canon(s_mul(r[c], f));
            f = s_canon(s_mul(f, step));
        }
    }
}

void canon_all(uint64_t *x, uint64_t m)
{
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < m; i++) x[i] = s_canon(x[i]);
}

// ---------------------------------------------------------------- Steps programs
// The reference evaluates its Steps bytecode 4 rows at a time with AVX2 (one
// case per op, zkevm.chelpers.step42ns.parser.cpp:24-784, Goldilocks3 *_avx
// helpers).  The same over the ZXP form of a program (include/zkgpu_zxp.h),
// with the oracle interpreter's semantics (oracle/stark.c zxp_run): every row
// starts with zero temporaries, a base operand of an extension add / sub is
// component 0, row shifts wrap mod the domain, stores are canonical.
struct V3 {
    V v[3];
    int dim;
};

struct ZEnv {
    uint64_t **sec;
    const uint64_t *stride;
    uint64_t dom;
    const uint64_t *challenges, *publics, *evals, *x, *xdiv, *xdivw, *zhinv;
    uint64_t zmask;
};

struct zop {
    uint32_t kind, a, b, c;
};
struct zin {
    uint32_t op, dst, a, b;
};

inline V gather_rows(const uint64_t *base, uint64_t stride, const uint64_t row[4])
{
    return _mm256_set_epi64x((long long)base[row[3] * stride], (long long)base[row[2] * stride],
                             (long long)base[row[1] * stride], (long long)base[row[0] * stride]);
}

inline V3 zload(const ZEnv &e, const zop &o, const V *t1, const V *t3, uint64_t i0, const uint64_t lane_row[4])
{
    V3 r;
    r.dim = 1;
    r.v[1] = r.v[2] = _mm256_setzero_si256();
    switch (o.kind) {
    case 0: r.v[0] = t1[o.a]; break;  // ZXP_TMP1
    case 1:                           // ZXP_TMP3
        r.v[0] = t3[3 * o.a];
        r.v[1] = t3[3 * o.a + 1];
        r.v[2] = t3[3 * o.a + 2];
        r.dim = 3;
        break;
    case 2:
    case 3: {  // ZXP_COL / COL3
        uint64_t row[4];
        const uint64_t sh = (uint64_t)(int64_t)(int32_t)o.c;
        for (int l = 0; l < 4; l++) row[l] = (lane_row[l] + sh + e.dom) % e.dom;
        const uint64_t *p = e.sec[o.a] + o.b;
        r.v[0] = v_canon(gather_rows(p, e.stride[o.a], row));
        if (o.kind == 3) {
            r.v[1] = v_canon(gather_rows(p + 1, e.stride[o.a], row));
            r.v[2] = v_canon(gather_rows(p + 2, e.stride[o.a], row));
            r.dim = 3;
        }
        break;
    }
    case 4: r.v[0] = bc(s_canon((uint64_t)o.a | ((uint64_t)o.b << 32))); break;  // LIT
    case 5:                                                                      // CHAL
    case 8:                                                                      // EVAL
    {
        const uint64_t *c = (o.kind == 5 ? e.challenges : e.evals) + 3 * o.a;
        for (int k = 0; k < 3; k++) r.v[k] = bc(s_canon(c[k]));
        r.dim = 3;
        break;
    }
    case 6: r.v[0] = bc(s_canon(e.publics[o.a])); break;   // PUB
    case 7: r.v[0] = v_canon(gather_rows(e.x, 1, lane_row)); break;  // X
    case 9:
    case 10: {  // XDIV / XDIVW (interleaved, 3 per row)
        const uint64_t *b = o.kind == 9 ? e.xdiv : e.xdivw;
        for (int k = 0; k < 3; k++) r.v[k] = v_canon(gather_rows(b + k, 3, lane_row));
        r.dim = 3;
        break;
    }
    case 11: {  // ZI
        uint64_t zr[4];
        for (int l = 0; l < 4; l++) zr[l] = lane_row[l] & e.zmask;
        r.v[0] = v_canon(gather_rows(e.zhinv, 1, zr));
        break;
    }
    default: r.v[0] = _mm256_setzero_si256(); break;
    }
    (void)i0;
    return r;
}

inline V3 zbinop(uint32_t op, const V3 &a, const V3 &b)
{
    V3 r;
    r.dim = (a.dim == 3 || b.dim == 3) ? 3 : 1;
    if (op == 2) {  // MUL
        if (a.dim == 3 && b.dim == 3) {
            // (a0 + a1 X + a2 X^2)(b0 + b1 X + b2 X^2), X^3 = X + 1 (polinomial.hpp:195-205)
            const V p0 = v_canon(v_mul(a.v[0], b.v[0])), p1 = v_canon(v_mul(a.v[1], b.v[1])),
                    p2 = v_canon(v_mul(a.v[2], b.v[2]));
            const V q01 = v_canon(v_mul(v_canon(v_add(a.v[0], a.v[1])), v_canon(v_add(b.v[0], b.v[1]))));
            const V q02 = v_canon(v_mul(v_canon(v_add(a.v[0], a.v[2])), v_canon(v_add(b.v[0], b.v[2]))));
            const V q12 = v_canon(v_mul(v_canon(v_add(a.v[1], a.v[2])), v_canon(v_add(b.v[1], b.v[2]))));
            const V c1 = v_canon(v_sub(v_canon(v_sub(q01, p0)), p1));
            const V c2 = v_canon(v_add(v_canon(v_sub(v_canon(v_sub(q02, p0)), p2)), p1));
            const V c3 = v_canon(v_sub(v_canon(v_sub(q12, p1)), p2));
            r.v[0] = v_canon(v_add(p0, c3));
            r.v[1] = v_canon(v_add(v_canon(v_add(c1, p2)), c3));
            r.v[2] = v_canon(v_add(c2, p2));
        } else if (a.dim == 3 || b.dim == 3) {
            const V3 &x = a.dim == 3 ? a : b;
            const V s = a.dim == 3 ? b.v[0] : a.v[0];
            for (int k = 0; k < 3; k++) r.v[k] = v_canon(v_mul(x.v[k], s));
        } else {
            r.v[0] = v_canon(v_mul(a.v[0], b.v[0]));
            r.v[1] = r.v[2] = _mm256_setzero_si256();
        }
        return r;
    }
    for (int k = 0; k < 3; k++) {
        const V av = (k == 0 || a.dim == 3) ? a.v[k] : _mm256_setzero_si256();
        const V bv = (k == 0 || b.dim == 3) ? b.v[k] : _mm256_setzero_si256();
        r.v[k] = v_canon(op == 0 ? v_add(av, bv) : v_sub(av, bv));
    }
    return r;
}

inline void zstore(const ZEnv &e, const zop &o, V *t1, V *t3, const V3 &v, const uint64_t lane_row[4], int nvalid)
{
    switch (o.kind) {
    case 0: t1[o.a] = v.v[0]; break;
    case 1:
        t3[3 * o.a] = v.v[0];
        t3[3 * o.a + 1] = v.dim == 3 ? v.v[1] : _mm256_setzero_si256();
        t3[3 * o.a + 2] = v.dim == 3 ? v.v[2] : _mm256_setzero_si256();
        break;
    case 2:
    case 3: {
        alignas(32) uint64_t c[3][4];
        for (int k = 0; k < 3; k++) _mm256_store_si256((V *)c[k], v.v[k]);
        const uint64_t sh = (uint64_t)(int64_t)(int32_t)o.c;
        for (int l = 0; l < nvalid; l++) {
            const uint64_t row = (lane_row[l] + sh + e.dom) % e.dom;
            uint64_t *p = e.sec[o.a] + row * e.stride[o.a] + o.b;
            p[0] = c[0][l];
            if (o.kind == 3) {
                p[1] = v.dim == 3 ? c[1][l] : 0;
                p[2] = v.dim == 3 ? c[2][l] : 0;
            }
        }
        break;
    }
    default: break;
    }
}

}  // namespace

extern "C" {

// oc_zxp_eval's contract (oracle/oracle.h), 4 rows per vector step
void cr_zxp_eval(const void *instr_v, uint32_t n_instr, const void *opnd_v, uint32_t n_tmp1, uint32_t n_tmp3,
                 uint64_t **sec, const uint64_t *stride, uint64_t dom, const uint64_t *challenges,
                 const uint64_t *publics, const uint64_t *evals, const uint64_t *x, const uint64_t *xdiv,
                 const uint64_t *xdivw, const uint64_t *zhinv, uint64_t zhinv_size)
{
    const zin *ins = (const zin *)instr_v;
    const zop *opn = (const zop *)opnd_v;
    const ZEnv e{sec, stride, dom, challenges, publics, evals, x, xdiv, xdivw, zhinv, zhinv_size ? zhinv_size - 1 : 0};
#pragma omp parallel
    {
        V *t1 = (V *)aligned_alloc(32, 32 * ((size_t)n_tmp1 + 1));
        V *t3 = (V *)aligned_alloc(32, 32 * (3 * (size_t)n_tmp3 + 3));
#pragma omp for schedule(static)
        for (uint64_t i0 = 0; i0 < dom; i0 += 4) {
            const int nvalid = dom - i0 < 4 ? (int)(dom - i0) : 4;
            uint64_t lane_row[4];
            for (int l = 0; l < 4; l++) lane_row[l] = i0 + (l < nvalid ? l : 0);
            memset((void *)t1, 0, 32 * ((size_t)n_tmp1 + 1));
            memset((void *)t3, 0, 32 * (3 * (size_t)n_tmp3 + 3));
            for (uint32_t k = 0; k < n_instr; k++) {
                const zin &in = ins[k];
                const V3 a = zload(e, opn[in.a], t1, t3, i0, lane_row);
                V3 r;
                if (in.op == 3) {
                    r = a;
                } else {
                    const V3 b = zload(e, opn[in.b], t1, t3, i0, lane_row);
                    r = zbinop(in.op, a, b);
                }
                zstore(e, opn[in.dst], t1, t3, r, lane_row, nvalid);
            }
        }
        free(t1);
        free(t3);
    }
}

void cr_set_num_threads(int n) { omp_set_num_threads(n); }
int cr_num_threads(void) { return omp_get_max_threads(); }

uint64_t cr_merkle_num_elements(uint64_t nrows) { return nrows ? 4 * nrows + 4 * (nrows - 1) : 0; }

// MerkleTreeGL::merkelize / PoseidonGoldilocks::merkletree_avx
// (merkleTreeGL.cpp:37-44, hpp:58-61): nodes = the leaf digests, then each
// level appended (node = hash(L || R || 0^4)[0..3]), root last; heights are
// powers of two in every reference use
void cr_merkletree(uint64_t *nodes, const uint64_t *src, uint64_t ncols, uint64_t nrows)
{
    if (!nrows) return;
#pragma omp parallel for schedule(dynamic, 64)
    for (uint64_t r0 = 0; r0 < nrows; r0 += 4) leaves4(nodes, src, ncols, r0, nrows - r0 < 4 ? nrows - r0 : 4);
    uint64_t off = 0, pending = nrows;
    while (pending > 1) {
        const uint64_t next = pending / 2;
        const uint64_t *cur = nodes + off;
        uint64_t *dst = nodes + off + 4 * pending;
#pragma omp parallel for schedule(static) if (next > 256)
        for (uint64_t p0 = 0; p0 < next; p0 += 4) nodes4(dst, cur, p0, next - p0 < 4 ? next - p0 : 4);
        off += 4 * pending;
        pending = next;
    }
}

void cr_ntt(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols, int inverse)
{
    if (!n || !ncols) return;
    const unsigned L = log2u(n);
    uint64_t root = s_w(L);
    if (inverse) root = s_pow(root, P - 2);
    if (dst == src) {
        uint64_t *tmp = (uint64_t *)malloc(8 * n * ncols);
        memcpy(tmp, src, 8 * n * ncols);
        bitrev_rows(dst, tmp, n, ncols);
        free(tmp);
    } else {
        bitrev_rows(dst, src, n, ncols);
    }
    dit(dst, n, ncols, root);
    if (inverse)
        scale_rows(dst, n, ncols, s_pow(n % P, P - 2), 1);
    else
        canon_all(dst, n * ncols);
}

// extendPol (starks.cpp:53): INTT_n, row i times shift^i / n, zero-pad, NTT_{n_ext}
void cr_extend_pol(uint64_t *out, const uint64_t *in, uint64_t n_ext, uint64_t n, uint64_t ncols)
{
    if (!n || !ncols) return;
    uint64_t *coef = (uint64_t *)malloc(8 * n * ncols);
    bitrev_rows(coef, in, n, ncols);
    dit(coef, n, ncols, s_pow(s_w(log2u(n)), P - 2));
    scale_rows(coef, n, ncols, s_pow(n % P, P - 2), 7);
    // zero-padded coefficients, bit-reversed into out, then the DIT
    const unsigned Le = log2u(n_ext);
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < n_ext; i++) {
        const uint64_t r = bitrev(i, Le);
        uint64_t *d = out + i * ncols;
        if (r < n)
            memcpy(d, coef + r * ncols, 8 * ncols);
        else
            memset(d, 0, 8 * ncols);
    }
    free(coef);
    dit(out, n_ext, ncols, s_w(Le));
    canon_all(out, n_ext * ncols);
}

}  // extern "C"
