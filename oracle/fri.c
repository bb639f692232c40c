/*
 * oracle/fri.c -- TEST INFRASTRUCTURE ONLY (CPU oracle).
 *
 * FRI fold restated from src/starkpil/fri/friProve.cpp:20-108 (si > 0 branch):
 *   for g < 2^out_bits:
 *     ppar[i]  = pol[i * 2^out_bits + g],  i < nX = 2^(pol_bits - out_bits)
 *     ppar_c   = INTT_nX(ppar)                                   (:102)
 *     ppar_c[i] *= (shiftInv * w(pol_bits)^-g)^i                 (polMulAxi :103, :183-191)
 *     out[g]   = Horner(ppar_c, special_x)                        (evalPol :104, :192-207)
 * getTransposed: friProve.cpp:252-270.
 */
#include <stdlib.h>
#include <string.h>
#include "gl.h"
#include "oracle.h"

void oc_fri_fold_group(uint64_t out[3], const uint64_t *vals, uint64_t nx, uint64_t g,
                       uint64_t pol_bits, const uint64_t special_x[3], uint64_t shift_inv)
{
    uint64_t *c = (uint64_t *)malloc(sizeof(uint64_t) * 3 * nx);
    oc_ntt(c, vals, nx, 3, 1);
    uint64_t wi = gl_inv(gl_w((unsigned)pol_bits));
    uint64_t sinv = gl_mul(shift_inv, gl_pow(wi, g));
    uint64_t r = 1;
    for (uint64_t i = 0; i < nx; i++) {
        gl3_mul1(c + 3 * i, c + 3 * i, r);
        r = gl_mul(r, sinv);
    }
    uint64_t acc[3];
    memcpy(acc, c + 3 * (nx - 1), sizeof acc);
    for (int64_t i = (int64_t)nx - 2; i >= 0; i--) {
        gl3_mul(acc, acc, special_x);
        gl3_add(acc, acc, c + 3 * i);
    }
    memcpy(out, acc, sizeof acc);
    free(c);
}

void oc_fri_fold(uint64_t *out, const uint64_t *pol, uint64_t pol_bits, uint64_t out_bits,
                 const uint64_t special_x[3], uint64_t shift_inv)
{
    uint64_t n_out = 1ULL << out_bits;
    uint64_t nx = 1ULL << (pol_bits - out_bits);
#pragma omp parallel for schedule(static)
    for (uint64_t g = 0; g < n_out; g++) {
        uint64_t vals[3 * 64];
        uint64_t *v = nx <= 64 ? vals : (uint64_t *)malloc(sizeof(uint64_t) * 3 * nx);
        for (uint64_t i = 0; i < nx; i++) memcpy(v + 3 * i, pol + 3 * (i * n_out + g), 3 * sizeof(uint64_t));
        oc_fri_fold_group(out + 3 * g, v, nx, g, pol_bits, special_x, shift_inv);
        if (v != vals) free(v);
    }
}

void oc_fri_get_transposed(uint64_t *aux, const uint64_t *pol, uint64_t degree, uint64_t transpose_bits)
{
    uint64_t w = 1ULL << transpose_bits;
    uint64_t h = degree / w;
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < w; i++)
        for (uint64_t j = 0; j < h; j++) memcpy(aux + 3 * (i * h + j), pol + 3 * (j * w + i), 3 * sizeof(uint64_t));
}
