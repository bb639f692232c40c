/*
 * oracle/ntt.c -- TEST INFRASTRUCTURE ONLY (CPU oracle + CPU baseline).
 *
 * Goldilocks NTT / INTT / extendPol on row-major buffers (n rows x ncols).
 * Restates the semantics of NTT_Goldilocks from the absent submodule as used
 * at starks.cpp:53,134,215 (extendPol), starks.cpp:262,285,326-327 (NTT/INTT)
 * and friProve.cpp:100-102 (16-point INTT), with the algorithm of the
 * reference's in-mount restatement tools/starkpil/bctree/build_const_tree.cpp:
 *   - bit-reverse the input (bitReverse, :275-283),
 *   - radix-2 decimation-in-time butterflies, first the stages whose span fits
 *     a cache block, per block in parallel (_fft_block, :216-262), then the
 *     remaining stages across the whole column set,
 *   - INTT = DFT with omega^-1 followed by the 1/n scale, and
 *   - extendPol = INTT_n, multiply row i by shift^i (interpolatePrepare,
 *     :320-345 folds the 1/n into the same factor), zero-pad, NTT_{n_ext}.
 */
#include <stdlib.h>
#include <string.h>
#include <omp.h>
#include "gl.h"
#include "oracle.h"

static unsigned log2u(uint64_t n)
{
    unsigned l = 0;
    while ((1ULL << l) < n) l++;
    return l;
}

static uint64_t bitrev(uint64_t x, unsigned bits)
{
    uint64_t r = 0;
    for (unsigned i = 0; i < bits; i++) {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

#define BLOCK_BITS 12

static void dit_core(uint64_t *x, uint64_t n, uint64_t ncols, uint64_t root)
{
    unsigned L = log2u(n);
    if (L == 0) return;
    uint64_t half_n = n >> 1;
    uint64_t *tw = (uint64_t *)malloc(sizeof(uint64_t) * (half_n ? half_n : 1));
    /* tw[k] = root^k, built in parallel chunks */
#pragma omp parallel for schedule(static)
    for (uint64_t c = 0; c < half_n; c += 4096) {
        uint64_t v = gl_pow(root, c);
        uint64_t end = c + 4096 < half_n ? c + 4096 : half_n;
        for (uint64_t k = c; k < end; k++) {
            tw[k] = v;
            v = gl_mul(v, root);
        }
    }
    unsigned B = L < BLOCK_BITS ? L : BLOCK_BITS;
    uint64_t bsz = 1ULL << B;
    /* stages 1..B inside blocks of bsz rows */
#pragma omp parallel for schedule(static)
    for (uint64_t blk = 0; blk < n; blk += bsz) {
        for (unsigned s = 1; s <= B; s++) {
            uint64_t half = 1ULL << (s - 1);
            uint64_t span = half << 1;
            uint64_t tstride = n >> s;
            for (uint64_t b = blk; b < blk + bsz; b += span) {
                for (uint64_t i = 0; i < half; i++) {
                    uint64_t w = tw[i * tstride];
                    uint64_t *u = x + (b + i) * ncols;
                    uint64_t *v = x + (b + i + half) * ncols;
                    for (uint64_t c = 0; c < ncols; c++) {
                        uint64_t t = gl_mul(v[c], w);
                        uint64_t a = u[c];
                        u[c] = gl_add(a, t);
                        v[c] = gl_sub(a, t);
                    }
                }
            }
        }
    }
    /* remaining stages across blocks */
    for (unsigned s = B + 1; s <= L; s++) {
        uint64_t half = 1ULL << (s - 1);
        uint64_t tstride = n >> s;
#pragma omp parallel for schedule(static)
        for (uint64_t k = 0; k < half_n; k++) {
            uint64_t i = k & (half - 1);
            uint64_t b = (k >> (s - 1)) << s;
            uint64_t w = tw[i * tstride];
            uint64_t *u = x + (b + i) * ncols;
            uint64_t *v = x + (b + i + half) * ncols;
            for (uint64_t c = 0; c < ncols; c++) {
                uint64_t t = gl_mul(v[c], w);
                uint64_t a = u[c];
                u[c] = gl_add(a, t);
                v[c] = gl_sub(a, t);
            }
        }
    }
    free(tw);
}

static void bitrev_copy(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols)
{
    unsigned L = log2u(n);
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < n; i++) {
        uint64_t r = bitrev(i, L);
        const uint64_t *s = src + r * ncols;
        uint64_t *d = dst + i * ncols;
        for (uint64_t c = 0; c < ncols; c++) d[c] = gl_canon(s[c]);
    }
}

void oc_ntt(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols, int inverse)
{
    if (n == 0 || ncols == 0) return;
    unsigned L = log2u(n);
    uint64_t root = gl_w(L);
    if (inverse) root = gl_inv(root);
    if (dst == src) {
        uint64_t *tmp = (uint64_t *)malloc(sizeof(uint64_t) * n * ncols);
        memcpy(tmp, src, sizeof(uint64_t) * n * ncols);
        bitrev_copy(dst, tmp, n, ncols);
        free(tmp);
    } else {
        bitrev_copy(dst, src, n, ncols);
    }
    dit_core(dst, n, ncols, root);
    if (inverse) {
        uint64_t ninv = gl_inv(n);
#pragma omp parallel for schedule(static)
        for (uint64_t i = 0; i < n * ncols; i++) dst[i] = gl_mul(dst[i], ninv);
    }
}

void oc_dft_naive(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols, int inverse)
{
    unsigned L = log2u(n);
    uint64_t root = gl_w(L);
    if (inverse) root = gl_inv(root);
    uint64_t ninv = inverse ? gl_inv(n) : 1;
    uint64_t *out = (uint64_t *)malloc(sizeof(uint64_t) * n * ncols);
    for (uint64_t k = 0; k < n; k++) {
        uint64_t wk = gl_pow(root, k);
        for (uint64_t c = 0; c < ncols; c++) {
            uint64_t acc = 0, w = 1;
            for (uint64_t j = 0; j < n; j++) {
                acc = gl_add(acc, gl_mul(src[j * ncols + c], w));
                w = gl_mul(w, wk);
            }
            out[k * ncols + c] = gl_mul(acc, ninv);
        }
    }
    memcpy(dst, out, sizeof(uint64_t) * n * ncols);
    free(out);
}

void oc_extend_pol(uint64_t *out, const uint64_t *in, uint64_t n_ext, uint64_t n, uint64_t ncols)
{
    if (n == 0 || ncols == 0) return;
    /* coefficients into the first n rows of out */
    oc_ntt(out, in, n, ncols, 1);
    /* r_i = shift^i  (INTT already applied 1/n) */
#pragma omp parallel for schedule(static)
    for (uint64_t c0 = 0; c0 < n; c0 += 4096) {
        uint64_t r = gl_pow(GL_SHIFT, c0);
        uint64_t end = c0 + 4096 < n ? c0 + 4096 : n;
        for (uint64_t i = c0; i < end; i++) {
            uint64_t *row = out + i * ncols;
            for (uint64_t c = 0; c < ncols; c++) row[c] = gl_mul(row[c], r);
            r = gl_mul(r, GL_SHIFT);
        }
    }
    memset(out + n * ncols, 0, sizeof(uint64_t) * (n_ext - n) * ncols);
    oc_ntt(out, out, n_ext, ncols, 0);
}

/* ---- exported scalar helpers ---- */
uint64_t oc_gl_mul(uint64_t a, uint64_t b) { return gl_mul(a, b); }
uint64_t oc_gl_add(uint64_t a, uint64_t b) { return gl_add(a, b); }
uint64_t oc_gl_sub(uint64_t a, uint64_t b) { return gl_sub(a, b); }
uint64_t oc_gl_inv(uint64_t a) { return gl_inv(a); }
uint64_t oc_gl_pow(uint64_t a, uint64_t e) { return gl_pow(a, e); }
uint64_t oc_gl_w(unsigned n) { return gl_w(n); }
void oc_gl3_mul(uint64_t *o, const uint64_t *a, const uint64_t *b) { gl3_mul(o, a, b); }
void oc_gl3_inv(uint64_t *o, const uint64_t *a) { gl3_inv(o, a); }
/* out[k] = base^k in F_p^3, k < n (the xi powers of Starks::genProof's LEv /
   LpEv, starks.cpp:314-327) */
void oc_powers3(uint64_t *out, const uint64_t *base, uint64_t n)
{
    if (n == 0) return;
    out[0] = 1;
    out[1] = out[2] = 0;
    for (uint64_t k = 1; k < n; k++) gl3_mul(out + 3 * k, out + 3 * (k - 1), base);
}
int oc_num_threads(void) { return omp_get_max_threads(); }
void oc_set_num_threads(int n) { omp_set_num_threads(n); }

/* Polinomial::batchInverse (polinomial.hpp:698-720) on ext elements */
void oc_batch_inverse3(uint64_t *out, const uint64_t *in, uint64_t n)
{
    if (n == 0) return;
    uint64_t *tmp = (uint64_t *)malloc(sizeof(uint64_t) * 3 * n);
    memcpy(tmp, in, 3 * sizeof(uint64_t));
    for (uint64_t i = 1; i < n; i++) gl3_mul(tmp + 3 * i, tmp + 3 * (i - 1), in + 3 * i);
    uint64_t z[3], z1[3];
    gl3_inv(z, tmp + 3 * (n - 1));
    for (uint64_t i = n - 1; i > 0; i--) {
        gl3_mul(z1, z, in + 3 * i);
        gl3_mul(out + 3 * i, z, tmp + 3 * (i - 1));
        memcpy(z, z1, sizeof z);
    }
    memcpy(out, z, sizeof z);
    free(tmp);
}
