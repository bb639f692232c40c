/*
 * oracle/transcript.c -- TEST INFRASTRUCTURE ONLY (CPU oracle).
 *
 * Fiat-Shamir transcript, restated from src/starkpil/transcript/transcript.cpp:4-87
 * (sponge: 8 pending + 4 state lanes into hash_full_result, squeeze
 * out[(12 - cursor) % 12], any put resets the squeeze cursor) and
 * getPermutations (:57-87: floor((n*nBits-1)/63)+1 squeezed fields, 63 usable
 * bits each, read LSB first).
 */
#include <string.h>
#include "gl.h"
#include "oracle.h"

void oc_transcript_init(oc_transcript *t) { memset(t, 0, sizeof *t); }

static void absorb(oc_transcript *t)
{
    uint64_t in[12];
    memcpy(in, t->pending, 8 * sizeof(uint64_t));
    memcpy(in + 8, t->state, 4 * sizeof(uint64_t));
    oc_poseidon_full(t->out, in);
    t->out_cursor = 12;
    memset(t->pending, 0, sizeof t->pending);
    t->pending_cursor = 0;
    memcpy(t->state, t->out, 4 * sizeof(uint64_t));
}

void oc_transcript_put(oc_transcript *t, const uint64_t *in, uint64_t n)
{
    for (uint64_t i = 0; i < n; i++) {
        t->pending[t->pending_cursor++] = in[i];
        t->out_cursor = 0;
        if (t->pending_cursor == 8) absorb(t);
    }
}

uint64_t oc_transcript_get_fields1(oc_transcript *t)
{
    if (t->out_cursor == 0) absorb(t);
    uint64_t r = t->out[(12 - t->out_cursor) % 12];
    t->out_cursor--;
    return r;
}

void oc_transcript_get_field(oc_transcript *t, uint64_t out[3])
{
    for (int i = 0; i < 3; i++) out[i] = oc_transcript_get_fields1(t);
}

void oc_transcript_get_permutations(oc_transcript *t, uint64_t *res, uint64_t n, uint64_t nbits)
{
    uint64_t total = n * nbits;
    uint64_t nfields = (total - 1) / 63 + 1;
    uint64_t fields[nfields];
    for (uint64_t i = 0; i < nfields; i++) fields[i] = gl_canon(oc_transcript_get_fields1(t));
    uint64_t cur_field = 0, cur_bit = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t a = 0;
        for (uint64_t j = 0; j < nbits; j++) {
            uint64_t bit = (fields[cur_field] >> cur_bit) & 1;
            if (bit) a += 1ULL << j;
            if (++cur_bit == 63) {
                cur_bit = 0;
                cur_field++;
            }
        }
        res[i] = a;
    }
}
