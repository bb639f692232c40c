/*
 * oracle/h1h2.c -- TEST INFRASTRUCTURE (CPU oracle; never linked into the
 * product).  Plookup h1/h2 columns, Polinomial::calculateH1H2_opt1 (dim 1,
 * polinomial.hpp:349-463) and calculateH1H2_opt3 (dim 3, :465-583), as called
 * from Starks::genProof stage 2 (starks.cpp:104-127).
 *
 * Semantics restated from the reference:
 *   - every table row j starts with multiplicity 1 (vector<int> counter(N, 1));
 *   - each f row adds 1 to the multiplicity of the LAST table row holding the
 *     same value (the hash chain stores the latest index, :380-383);
 *     all dim components are compared canonically (toU64 / toVectorU64);
 *   - the sorted multiset s = t[0]^c0 t[1]^c1 ... (length 2N) is dealt
 *     alternately: h1[i] = s[2i], h2[i] = s[2i+1] (:443-462);
 *   - an f value absent from t is an error ("Number not included", the
 *     reference logs and exits): returns 1 + the first such f row, else 0.
 * Rows are `stride` u64 apart (row-major sections, stark_info.cpp:473-482).
 * The hash table is replaced by a sort + binary search: same mapping.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gl.h"
#include "oracle.h"

typedef struct {
    uint64_t k[3];
    uint64_t idx;
} h12_ent;

static int h12_dim;

static int cmp_key(const uint64_t *a, const uint64_t *b, int dim)
{
    for (int c = 0; c < dim; c++) {
        if (a[c] < b[c]) return -1;
        if (a[c] > b[c]) return 1;
    }
    return 0;
}

static int cmp_ent(const void *x, const void *y)
{
    const h12_ent *a = (const h12_ent *)x, *b = (const h12_ent *)y;
    int r = cmp_key(a->k, b->k, h12_dim);
    if (r) return r;
    return a->idx < b->idx ? -1 : (a->idx > b->idx ? 1 : 0);
}

uint64_t oc_h1h2(uint64_t *h1, uint64_t h1s, uint64_t *h2, uint64_t h2s, const uint64_t *f, uint64_t fs,
                 const uint64_t *t, uint64_t ts, uint64_t n, uint32_t dim)
{
    h12_ent *e = (h12_ent *)malloc(n * sizeof(h12_ent));
    uint64_t *cnt = (uint64_t *)malloc(n * sizeof(uint64_t));
    uint64_t missing = 0;
    for (uint64_t i = 0; i < n; i++) {
        e[i].k[0] = e[i].k[1] = e[i].k[2] = 0;
        for (uint32_t c = 0; c < dim; c++) e[i].k[c] = gl_canon(t[i * ts + c]);
        e[i].idx = i;
        cnt[i] = 1;
    }
    h12_dim = (int)dim;
    qsort(e, n, sizeof(h12_ent), cmp_ent);
    for (uint64_t i = 0; i < n && !missing; i++) {
        uint64_t key[3] = {0, 0, 0};
        for (uint32_t c = 0; c < dim; c++) key[c] = gl_canon(f[i * fs + c]);
        /* upper bound of key, then step back: the last (highest index) table row */
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            uint64_t mid = (lo + hi) / 2;
            if (cmp_key(e[mid].k, key, (int)dim) <= 0) lo = mid + 1;
            else hi = mid;
        }
        if (lo == 0 || cmp_key(e[lo - 1].k, key, (int)dim) != 0) {
            missing = i + 1;
            break;
        }
        cnt[e[lo - 1].idx]++;
    }
    if (!missing) {
        uint64_t id = 0;
        for (uint64_t i = 0; i < n; i++) {
            if (cnt[id] == 0) id++;
            cnt[id]--;
            for (uint32_t c = 0; c < dim; c++) h1[i * h1s + c] = t[id * ts + c];
            if (cnt[id] == 0) id++;
            cnt[id]--;
            for (uint32_t c = 0; c < dim; c++) h2[i * h2s + c] = t[id * ts + c];
        }
    }
    free(e);
    free(cnt);
    return missing;
}
