/*
 * oracle/poseidon.c -- TEST INFRASTRUCTURE ONLY (CPU oracle).
 *
 * Poseidon-GL permutation in its plain (non-sparse) textbook form, restated
 * from the reference's own scalar implementation
 * src/sm/poseidon_g/poseidon_g_executor.cpp:201-231 (round loop) and
 * poseidon_g_executor.hpp:29-51 (t=12, RF=8, RP=22, MCIRC/MDIAG matrix):
 *   per round r: state += C[12r..12r+11]; S-box x^7 on all lanes for the
 *   4 first and 4 last rounds, on lane 0 only for the 22 middle rounds;
 *   state' = M * state with M[i][j] = MCIRC[(j-i) mod 12] + (i==j)*MDIAG[i].
 * hash_full_result returns all 12 lanes, hash the first 4 (transcript.cpp:23).
 * linear_hash is the sponge of SURVEY.md 8(a) a6 (submodule, absent):
 * <= 4 inputs are copied and zero-padded; otherwise chunks of 8 into lanes
 * 0..7 (last chunk zero-padded), capacity lanes 8..11 = 0 for the first chunk
 * and the previous output lanes 0..3 afterwards; digest = out lanes 0..3.
 */
#include <string.h>
#include "gl.h"
#include "oracle.h"
#include "poseidon_gl_constants.h"

static const uint64_t MCIRC[12] = {17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20};
static const uint64_t MDIAG[12] = {8, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

static inline uint64_t pow7(uint64_t x)
{
    uint64_t x2 = gl_mul(x, x);
    uint64_t x3 = gl_mul(x2, x);
    uint64_t x4 = gl_mul(x2, x2);
    return gl_mul(x3, x4);
}

void oc_poseidon_full(uint64_t out[12], const uint64_t in[12])
{
    uint64_t st[12];
    for (int i = 0; i < 12; i++) st[i] = gl_canon(in[i]);
    for (int r = 0; r < 30; r++) {
        for (int s = 0; s < 12; s++) st[s] = gl_add(st[s], ORACLE_POSEIDON_RC[r * 12 + s]);
        if (r < 4 || r >= 26) {
            for (int s = 0; s < 12; s++) st[s] = pow7(st[s]);
        } else {
            st[0] = pow7(st[0]);
        }
        uint64_t acc[12];
        for (int x = 0; x < 12; x++) {
            u128 a = 0;
            for (int y = 0; y < 12; y++) {
                uint64_t m = MCIRC[(y - x + 12) % 12] + (x == y ? MDIAG[x] : 0);
                a += (u128)st[y] * m;
            }
            acc[x] = gl_reduce128(a);
        }
        memcpy(st, acc, sizeof st);
    }
    memcpy(out, st, sizeof st);
}

void oc_poseidon_hash(uint64_t out[4], const uint64_t in[12])
{
    uint64_t full[12];
    oc_poseidon_full(full, in);
    memcpy(out, full, 4 * sizeof(uint64_t));
}

void oc_linear_hash(uint64_t out[4], const uint64_t *in, uint64_t size)
{
    if (size <= 4) {
        for (uint64_t i = 0; i < 4; i++) out[i] = i < size ? in[i] : 0;
        return;
    }
    uint64_t st[12];
    uint64_t remaining = size;
    while (remaining) {
        if (remaining == size) {
            memset(st + 8, 0, 4 * sizeof(uint64_t));
        } else {
            memcpy(st + 8, st, 4 * sizeof(uint64_t));
        }
        uint64_t n = remaining < 8 ? remaining : 8;
        memset(st + n, 0, (8 - n) * sizeof(uint64_t));
        memcpy(st, in + (size - remaining), n * sizeof(uint64_t));
        oc_poseidon_full(st, st);
        remaining -= n;
    }
    memcpy(out, st, 4 * sizeof(uint64_t));
}
