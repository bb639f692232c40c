/*
 * oracle/parser.c -- TEST INFRASTRUCTURE ONLY (CPU oracle).
 *
 * A scalar restatement of the reference's Steps bytecode interpreters, the
 * AVX2 `case` tables of
 *   src/starkpil/zkevm/chelpers/zkevm.chelpers.step2prev.parser.cpp:9-960
 *   src/starkpil/zkevm/chelpers/zkevm.chelpers.step3prev.parser.cpp:9-960
 *   src/starkpil/zkevm/chelpers/zkevm.chelpers.step3.parser.cpp:11-972
 *   src/starkpil/zkevm/chelpers/zkevm.chelpers.step42ns.parser.cpp:11-793
 *   src/starkpil/zkevm/chelpers/zkevm.chelpers.step52ns.parser.cpp:9-226
 * one row at a time (the reference runs 4 rows per AVX2 lane group; every
 * opcode is row-local except the shifted accesses written out below).
 *
 * Memory: the reference addresses one flat buffer, pols[off + row*stride]
 * (StepsParams.pols, the mapOffsets / mapSectionsN map, stark_info.cpp:473-482).
 * Here the caller passes the sections of that map it populated: an access
 * (off, stride) lands in the section whose stride matches and whose
 * [base, base + stride) contains off, at column off - base.  Shifted accesses
 * pols[off + ((i + s) % M) * stride] require M to be the circuit's domain
 * (native_dom) and wrap on the evaluated domain (dom rows), so the programs
 * can be checked on a smaller domain.  Constant pols: row-major, numpols wide.
 *
 * Field: Goldilocks; F_p^3 = F_p[x]/(x^3 - x - 1) (polinomial.hpp:195-205).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>
#include "gl.h"
#include "oracle.h"

typedef struct {
    uint32_t n_sec;
    const uint64_t *sec_off;    /* base offset of each section in the reference's map */
    const uint64_t *sec_stride; /* row stride (= width) */
    uint64_t *const *sec_ptr;   /* host row-major storage, dom rows */
    const uint64_t *cpols;      /* constant pols, row-major */
    uint64_t numpols;
    uint64_t dom, native_dom;
    const uint64_t *challenges, *publics, *evals, *x, *zhinv, *xdiv, *xdivw;
    uint64_t zhinv_mask;
    uint64_t *q, *f; /* dom x 3 outputs (step42ns / step52ns) */
    int err;
    /* sampled rows (oc_parser_eval_rows): every row-indexed array holds only
     * the rows rmap[0..nmap) (sorted), row r at index rix(r); NULL: all rows */
    const uint64_t *rmap;
    uint64_t nmap;
} penv;

static uint64_t rix(penv *e, uint64_t row)
{
    if (!e->rmap) return row;
    uint64_t lo = 0, hi = e->nmap;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (e->rmap[mid] < row) lo = mid + 1;
        else hi = mid;
    }
    if (lo == e->nmap || e->rmap[lo] != row) {
        e->err = 5; /* a row the caller did not provide */
        return 0;
    }
    return lo;
}

static uint64_t *mp(penv *e, uint64_t off, uint64_t row, uint64_t stride)
{
    for (uint32_t k = 0; k < e->n_sec; k++)
        if (e->sec_stride[k] == stride && off >= e->sec_off[k] && off < e->sec_off[k] + stride)
            return e->sec_ptr[k] + rix(e, row) * stride + (off - e->sec_off[k]);
    e->err = 1;
    static uint64_t sink[4];
    return sink;
}

static uint64_t srow(penv *e, uint64_t i, uint64_t s, uint64_t m)
{
    if (m != e->native_dom) e->err = 2;
    return (i + s) % e->dom;
}

/* F_p^3 helpers (outputs may alias inputs) */
static void a13(uint64_t *o, uint64_t a, const uint64_t *b)
{
    uint64_t r[3] = {gl_add(a, b[0]), b[1], b[2]};
    memcpy(o, r, 24);
}
static void a33(uint64_t *o, const uint64_t *a, const uint64_t *b)
{
    uint64_t r[3];
    gl3_add(r, a, b);
    memcpy(o, r, 24);
}
static void s33(uint64_t *o, const uint64_t *a, const uint64_t *b)
{
    uint64_t r[3];
    gl3_sub(r, a, b);
    memcpy(o, r, 24);
}
static void s31(uint64_t *o, const uint64_t *a, uint64_t b)
{
    uint64_t r[3] = {gl_sub(a[0], b), a[1], a[2]};
    memcpy(o, r, 24);
}
static void s13(uint64_t *o, uint64_t a, const uint64_t *b)
{
    uint64_t r[3] = {gl_sub(a, b[0]), gl_neg(b[1]), gl_neg(b[2])};
    memcpy(o, r, 24);
}
static void m13(uint64_t *o, uint64_t a, const uint64_t *b)
{
    uint64_t r[3];
    gl3_mul1(r, b, a);
    memcpy(o, r, 24);
}
static void m33(uint64_t *o, const uint64_t *a, const uint64_t *b)
{
    uint64_t r[3];
    gl3_mul(r, a, b);
    memcpy(o, r, 24);
}
static void st1(uint64_t *p, uint64_t v) { p[0] = gl_canon(v); }
static void st3(uint64_t *p, const uint64_t *v)
{
    p[0] = gl_canon(v[0]);
    p[1] = gl_canon(v[1]);
    p[2] = gl_canon(v[2]);
}

#define A(k) (args[ia + (k)])
#define T1(k) t1[A(k)]
#define T3(k) (t3 + 3 * A(k))
#define PP(o, s) mp(e, A(o), i, A(s))                          /* pols[a_o + i*a_s]             */
#define PSP(o, h, m, s) mp(e, A(o), srow(e, i, A(h), A(m)), A(s)) /* pols[a_o + ((i+a_h)%a_m)*a_s] */
#define PV(o, s) (*PP(o, s))
#define PSV(o, h, m, s) (*PSP(o, h, m, s))
#define KV(c) (e->cpols[rix(e, i) * e->numpols + A(c)])
#define KSV(c, h, m) (e->cpols[rix(e, srow(e, i, A(h), A(m))) * e->numpols + A(c)])
#define LV(k) (A(k))
#define CH(k) (e->challenges + 3 * A(k))
#define UV(k) (e->publics[A(k)])
#define XV (e->x[rix(e, i)])

/* opcodes 0..83, shared by step2prev / step3prev / step3 / step42ns (the
 * stage-3 parsers read x_n and constPols, step42ns x_2ns and constPols2ns:
 * the caller passes the matching x and constant pols).  Returns the argument
 * count, or -1 for an opcode outside this range. */
static int op_common(penv *e, uint64_t op, const uint64_t *args, uint64_t ia, uint64_t i, uint64_t *t1, uint64_t *t3)
{
    uint64_t w[3];
    switch (op) {
    case 0: T1(0) = gl_add(T1(1), T1(2)); return 3;
    case 1: T1(0) = gl_add(T1(1), PV(2, 3)); return 4;
    case 2: T1(0) = gl_add(T1(1), LV(2)); return 3;
    case 3: T1(0) = gl_add(T1(1), KV(2)); return 3;
    case 4: T1(0) = gl_add(PV(1, 2), PV(3, 4)); return 5;
    case 5: T1(0) = gl_add(PSV(1, 2, 3, 4), PSV(5, 6, 7, 8)); return 9;
    case 6: T1(0) = gl_add(PV(1, 2), KV(3)); return 4;
    case 7: T1(0) = gl_add(PV(1, 2), LV(3)); return 4;
    case 8: T1(0) = gl_add(KV(1), KV(2)); return 3;
    case 9: T1(0) = gl_add(KSV(1, 2, 3), KSV(4, 5, 6)); return 7;
    case 10: T1(0) = gl_add(KV(1), LV(2)); return 3;
    case 11: T1(0) = gl_add(KSV(1, 2, 3), LV(4)); return 5;
    case 12: a13(T3(0), T1(1), T3(2)); return 3;
    case 13: a13(T3(0), LV(1), CH(2)); return 3;
    case 14: a13(T3(0), T1(1), CH(2)); return 3;
    case 15: a13(T3(0), PV(1, 2), T3(3)); return 4;
    case 16: a13(T3(0), PV(1, 2), CH(3)); return 4;
    case 17: a33(T3(0), T3(1), T3(2)); return 3;
    case 18: a33(T3(0), T3(1), CH(2)); return 3;
    case 19: a33(T3(0), PP(1, 2), T3(3)); return 4;
    case 20: a33(T3(0), PP(1, 2), CH(3)); return 4;
    case 21: T1(0) = gl_sub(T1(1), T1(2)); return 3;
    case 22: T1(0) = gl_sub(T1(1), PV(2, 3)); return 4;
    case 23: T1(0) = gl_sub(T1(1), PSV(2, 3, 4, 5)); return 6;
    case 24: T1(0) = gl_sub(PV(1, 2), T1(3)); return 4;
    case 25: T1(0) = gl_sub(PSV(1, 2, 3, 4), T1(5)); return 6;
    case 26: T1(0) = gl_sub(T1(1), LV(2)); return 3;
    case 27: T1(0) = gl_sub(LV(1), T1(2)); return 3;
    case 28: T1(0) = gl_sub(PV(1, 2), LV(3)); return 4;
    case 29: T1(0) = gl_sub(PSV(1, 2, 3, 4), LV(5)); return 6;
    case 30: T1(0) = gl_sub(LV(1), PV(2, 3)); return 4;
    case 31: T1(0) = gl_sub(LV(1), PSV(2, 3, 4, 5)); return 6;
    case 32: T1(0) = gl_sub(LV(1), KV(2)); return 3;
    case 33: T1(0) = gl_sub(LV(1), KSV(2, 3, 4)); return 5;
    case 34: T1(0) = gl_sub(PV(1, 2), UV(3)); return 4;
    case 35: T1(0) = gl_sub(PSV(1, 2, 3, 4), PV(5, 6)); return 7;
    case 36: T1(0) = gl_sub(PV(1, 2), PSV(3, 4, 5, 6)); return 7;
    case 37: T1(0) = gl_sub(PV(1, 2), PV(3, 4)); return 5;
    case 38: T1(0) = gl_sub(PSV(1, 2, 3, 4), PSV(5, 6, 7, 8)); return 9;
    case 39: T1(0) = gl_sub(KV(1), PV(2, 3)); return 4;
    case 40: T1(0) = gl_sub(T1(1), KV(2)); return 3;
    case 41: s31(T3(0), PP(1, 2), LV(3)); return 4;
    case 42: s33(T3(0), T3(1), T3(2)); return 3;
    case 43: s33(T3(0), T3(1), CH(2)); return 3;
    case 44: s33(T3(0), T3(1), PP(2, 3)); return 4;
    case 45: T1(0) = gl_mul(T1(1), T1(2)); return 3;
    case 46: T1(0) = gl_mul(LV(1), T1(2)); return 3;
    case 47: T1(0) = gl_mul(PV(1, 2), T1(3)); return 4;
    case 48: T1(0) = gl_mul(PSV(1, 2, 3, 4), T1(5)); return 6;
    case 49: T1(0) = gl_mul(T1(1), KV(2)); return 3;
    case 50: T1(0) = gl_mul(PV(1, 2), PV(3, 4)); return 5;
    case 51: T1(0) = gl_mul(PV(1, 2), PSV(3, 4, 5, 6)); return 7;
    case 52: T1(0) = gl_mul(PSV(1, 2, 3, 4), PSV(5, 6, 7, 8)); return 9;
    case 53: T1(0) = gl_mul(LV(1), PV(2, 3)); return 4;
    case 54: T1(0) = gl_mul(PV(1, 2), KV(3)); return 4;
    case 55: T1(0) = gl_mul(PSV(1, 2, 3, 4), KV(5)); return 6;
    case 56: T1(0) = gl_mul(T1(1), PV(2, 3)); return 4;
    case 57: T1(0) = gl_mul(T1(1), PSV(2, 3, 4, 5)); return 6;
    case 58: T1(0) = gl_mul(KV(1), T1(2)); return 3;
    case 59: m13(T3(0), T1(1), CH(2)); return 3;
    case 60: m13(T3(0), KV(1), T3(2)); return 3;
    case 61: m13(T3(0), T1(1), T3(2)); return 3;
    case 62: m13(T3(0), PV(1, 2), CH(3)); return 4;
    case 63: m13(T3(0), PSV(1, 2, 3, 4), CH(5)); return 6;
    case 64: m13(T3(0), PV(1, 2), T3(3)); return 4;
    case 65: m13(T3(0), PSV(1, 2, 3, 4), T3(5)); return 6;
    case 66: m13(T3(0), LV(1), CH(2)); return 3;
    case 67: m13(T3(0), XV, CH(1)); return 2;
    case 68: m13(T3(0), XV, T3(1)); return 2;
    case 69: /* q_2ns[i] = zhInv(i) * tmp3 */
        if (!e->q) e->err = 3;
        else m13(e->q + 3 * rix(e, i), e->zhinv[i & e->zhinv_mask], T3(0));
        if (e->q) st3(e->q + 3 * rix(e, i), e->q + 3 * rix(e, i));
        return 1;
    case 70: m33(T3(0), T3(2), CH(1)); return 3;
    case 71: m33(T3(0), T3(1), T3(2)); return 3;
    case 72: m33(T3(0), PP(1, 2), PP(3, 4)); return 5;
    case 73: m33(T3(0), PSP(1, 2, 3, 4), CH(5)); return 6;
    case 74: m33(T3(0), PSP(1, 2, 3, 4), T3(5)); return 6;
    case 75: m33(T3(0), PP(1, 2), T3(3)); return 4;
    case 76: m33(T3(0), PP(1, 2), CH(3)); return 4;
    case 77: m33(T3(0), PSP(1, 2, 3, 4), PP(5, 6)); return 7;
    case 78: T1(0) = T1(1); return 2;
    case 79: T1(0) = PV(1, 2); return 3;
    case 80: T1(0) = PSV(1, 2, 3, 4); return 5;
    case 81: T1(0) = LV(1); return 2;
    case 82: T1(0) = KV(1); return 2;
    case 83: T1(0) = KSV(1, 2, 3); return 4;
    default: (void)w; return -1;
    }
}

/* step2prev / step3prev / step3 opcodes 84..120: stores into pols (rows i
 * and (i + s) % N) and a few fused forms (step3.parser.cpp:590-972) */
static int op_stage3(penv *e, uint64_t op, const uint64_t *args, uint64_t ia, uint64_t i, uint64_t *t1, uint64_t *t3)
{
    uint64_t w[3];
    switch (op) {
    case 84: T1(0) = gl_add(T1(1), PSV(2, 3, 4, 5)); return 6;
    case 85: T1(0) = gl_mul(PSV(1, 2, 3, 4), LV(5)); return 6;
    case 86: st1(PP(0, 1), gl_add(T1(2), T1(3))); return 4;
    case 87: st1(PP(0, 1), gl_add(T1(2), PV(3, 4))); return 5;
    case 88: a13(w, T1(2), T3(3)); st3(PP(0, 1), w); return 4;
    case 89: a33(w, PP(2, 3), T3(4)); st3(PP(0, 1), w); return 5;
    case 90: a33(w, T3(2), CH(3)); st3(PP(0, 1), w); return 4;
    case 91: st1(PP(0, 1), KV(2)); return 3;
    case 92: st1(PP(0, 1), gl_sub(T1(2), T1(3))); return 4;
    case 93: st1(PP(0, 1), gl_sub(LV(2), T1(3))); return 4;
    case 94: st1(PP(0, 1), gl_mul(T1(2), T1(3))); return 4;
    case 95: st1(PP(0, 1), gl_mul(PV(2, 3), T1(4))); return 5;
    case 96: st1(PP(0, 1), gl_mul(T1(2), KV(3))); return 4;
    case 97: s33(w, T3(2), T3(3)); st3(PP(0, 1), w); return 4;
    case 98: m33(w, T3(2), T3(3)); st3(PP(0, 1), w); return 4;
    case 99: st1(PP(0, 1), gl_mul(PV(2, 3), KV(4))); return 5;
    case 100: st1(PP(0, 1), T1(2)); return 3;
    /* shifted stores: pols[a0 + ((i + a1) % a2) * a3] */
    case 101: st1(PSP(0, 1, 2, 3), gl_add(T1(4), T1(5))); return 6;
    case 102: st1(PSP(0, 1, 2, 3), gl_add(T1(4), PV(5, 6))); return 7;
    case 103: a13(w, T1(4), T3(5)); st3(PSP(0, 1, 2, 3), w); return 6;
    case 104: a33(w, PP(4, 5), T3(6)); st3(PSP(0, 1, 2, 3), w); return 7;
    case 105: a33(w, T3(4), CH(5)); st3(PSP(0, 1, 2, 3), w); return 6;
    case 106: st1(PSP(0, 1, 2, 3), gl_sub(T1(4), T1(5))); return 6;
    case 107: st1(PSP(0, 1, 2, 3), gl_sub(LV(4), T1(5))); return 6;
    case 108: st1(PSP(0, 1, 2, 3), gl_mul(T1(4), T1(5))); return 6;
    case 109: st1(PSP(0, 1, 2, 3), gl_mul(PV(4, 5), T1(6))); return 7;
    case 110: st1(PSP(0, 1, 2, 3), gl_mul(T1(4), KV(5))); return 6;
    case 111: st1(PSP(0, 1, 2, 3), gl_mul(KSV(4, 5, 6), T1(7))); return 8;
    case 112: m33(w, T3(4), T3(5)); st3(PSP(0, 1, 2, 3), w); return 6;
    case 113: st1(PSP(0, 1, 2, 3), T1(4)); return 5;
    case 114: st1(PSP(0, 1, 2, 3), gl_add(T1(4), PSV(5, 6, 7, 8))); return 9;
    case 115: /* fused: 0 then 50 (step3 only) */
        T1(0) = gl_add(T1(1), T1(2));
        T1(3) = gl_mul(PV(4, 5), PV(6, 7));
        return 8;
    case 116: a33(w, T3(2), T3(3)); st3(PP(0, 1), w); return 4;
    case 117: st1(PP(0, 1), PV(2, 3)); return 4;
    case 118: st1(PP(0, 1), gl_add(PV(2, 3), PV(4, 5))); return 6;
    case 119: st1(PSP(0, 1, 2, 3), gl_mul(PSV(4, 5, 6, 7), KSV(8, 9, 10))); return 11;
    case 120: m33(w, PP(2, 3), T3(4)); st3(PP(0, 1), w); return 5;
    default: return -1;
    }
}

/* step42ns fused opcodes 84..92 (step42ns.parser.cpp:661-776): concatenations
 * of common opcodes over consecutive argument groups */
static int op_42ns(penv *e, uint64_t op, const uint64_t *args, uint64_t ia, uint64_t i, uint64_t *t1, uint64_t *t3)
{
    switch (op) {
    case 84: /* 12, 70 */
        a13(T3(0), T1(1), T3(2));
        m33(T3(3), T3(5), CH(4));
        return 6;
    case 85: /* 0, 50 */
        T1(0) = gl_add(T1(1), T1(2));
        T1(3) = gl_mul(PV(4, 5), PV(6, 7));
        return 8;
    case 86: /* 32, 47, 21, 32, 48 */
        T1(0) = gl_sub(LV(1), KV(2));
        T1(3) = gl_mul(PV(4, 5), T1(6));
        T1(7) = gl_sub(T1(8), T1(9));
        T1(10) = gl_sub(LV(11), KV(12));
        T1(13) = gl_mul(PSV(14, 15, 16, 17), T1(18));
        return 19;
    case 87: /* 4 x (12, 70) */
        for (int g = 0; g < 4; g++) {
            const uint64_t b = 6 * g;
            a13(t3 + 3 * A(b), t1[A(b + 1)], t3 + 3 * A(b + 2));
            m33(t3 + 3 * A(b + 3), t3 + 3 * A(b + 5), e->challenges + 3 * A(b + 4));
        }
        return 24;
    case 88: /* 21, 50, 21, 53, 0, 0, 50, 50, 0, 50, 21, 50 */
        T1(0) = gl_sub(T1(1), T1(2));
        T1(3) = gl_mul(PV(4, 5), PV(6, 7));
        T1(8) = gl_sub(T1(9), T1(10));
        T1(11) = gl_mul(LV(12), PV(13, 14));
        T1(15) = gl_add(T1(16), T1(17));
        T1(18) = gl_add(T1(19), T1(20));
        T1(21) = gl_mul(PV(22, 23), PV(24, 25));
        T1(26) = gl_mul(PV(27, 28), PV(29, 30));
        T1(31) = gl_add(T1(32), T1(33));
        T1(34) = gl_mul(PV(35, 36), PV(37, 38));
        T1(39) = gl_sub(T1(40), T1(41));
        T1(42) = gl_mul(PV(43, 44), PV(45, 46));
        return 47;
    case 89: s31(T3(0), PSP(1, 2, 3, 4), LV(5)); return 6;
    case 90: T1(0) = gl_mul(PSV(1, 2, 3, 4), KSV(5, 6, 7)); return 8;
    case 91: T1(0) = gl_sub(PV(1, 2), KV(3)); return 4;
    case 92: T1(0) = gl_sub(KV(1), T1(2)); return 3;
    default: return -1;
    }
}

/* step52ns (step52ns.parser.cpp:9-226): three F_p^3 accumulators T0, T1, T2
 * (T2 zero at the start of each row), v1 = challenges[5], v2 = challenges[6] */
static int op_52ns(penv *e, uint64_t op, const uint64_t *args, uint64_t ia, uint64_t i, uint64_t *acc)
{
    uint64_t *T0 = acc, *T1a = acc + 3, *T2 = acc + 6, w[3];
    const uint64_t *v1 = e->challenges + 15, *v2 = e->challenges + 18;
    const uint64_t *ev = e->evals;
    switch (op) {
    case 0: m13(T0, PV(0, 1), v1); return 2;
    case 1: m33(T0, T0, v1); return 0;
    case 2: m33(T0, T0, v2); return 0;
    case 3: m33(T1a, T0, v1); return 0;
    case 4: m33(T0, T2, v2); return 0;
    case 5: m33(T0, T0, e->xdiv + 3 * rix(e, i)); return 0;
    case 6: m33(T0, T0, e->xdivw + 3 * rix(e, i)); return 0;
    case 7: a33(T0, T0, T2); return 0;
    case 8: a33(T0, T1a, T0); return 0;
    case 9: a33(T0, T0, PP(0, 1)); return 2;
    case 10: a13(T0, PV(0, 1), T0); return 2;
    case 11: s13(T2, PV(0, 1), ev + 3 * A(2)); return 3;
    case 12: s33(T2, PP(0, 1), ev + 3 * A(2)); return 3;
    case 13: s13(T2, KV(0), ev + 3 * A(1)); return 2;
    case 14: s13(T0, e->cpols[rix(e, i) * e->numpols + 5], ev); return 0;
    case 15: st3(e->f + 3 * rix(e, i), T0); return 0;
    case 16: m33(T0, T0, v1); a13(T0, PV(0, 1), T0); return 2;
    case 17: m33(T0, T0, v1); a33(T0, T0, PP(0, 1)); return 2;
    case 18: m33(T0, T0, v2); s13(T2, PV(0, 1), ev + 3 * A(2)); a33(T0, T0, T2); return 3;
    case 19: m33(T0, T0, v2); s13(T2, KV(0), ev + 3 * A(1)); a33(T0, T0, T2); return 2;
    case 20: m33(T0, T0, v2); s33(T2, PP(0, 1), ev + 3 * A(2)); a33(T0, T0, T2); return 3;
    case 21: s13(T0, PV(0, 1), ev + 3 * A(2)); return 3;
    default: (void)w; return -1;
    }
}

/* the shared row loop: rows[0..n_rows) of the dom-row domain, or every row
 * (rows NULL); rmap / nmap as in penv */
static int parser_run(int parser, const uint64_t *ops, uint64_t n_ops, const uint64_t *args, uint64_t n_args,
                      uint32_t n_sec, const uint64_t *sec_off, const uint64_t *sec_stride, uint64_t *const *sec_ptr,
                      const uint64_t *cpols, uint64_t numpols, uint64_t dom, uint64_t native_dom, uint32_t n_tmp1,
                      uint32_t n_tmp3, const uint64_t *challenges, const uint64_t *publics, const uint64_t *evals,
                      const uint64_t *x, const uint64_t *zhinv, uint64_t zhinv_size, const uint64_t *xdiv,
                      const uint64_t *xdivw, uint64_t *q, uint64_t *f, const uint64_t *rows, uint64_t n_rows,
                      const uint64_t *rmap, uint64_t nmap)
{
    int status = 0;
    const uint64_t n_iter = rows ? n_rows : dom;
#pragma omp parallel
    {
        penv e = {n_sec,  sec_off, sec_stride, sec_ptr, cpols, numpols, dom,   native_dom, challenges, publics, evals,
                  x,      zhinv,   xdiv,       xdivw,   zhinv_size ? zhinv_size - 1 : 0,  q,     f,          0,
                  rmap,   nmap};
        uint64_t *t1 = (uint64_t *)calloc(n_tmp1 + 1, 8);
        uint64_t *t3 = (uint64_t *)calloc(3 * (uint64_t)n_tmp3 + 9, 8);
        int bad = 0;
#pragma omp for schedule(static)
        for (uint64_t it = 0; it < n_iter; it++) {
            if (bad) continue;
            const uint64_t i = rows ? rows[it] : it;
            uint64_t ia = 0;
            if (parser == 4) memset(t3, 0, 9 * 8); /* step52ns: tmp2 = 0 per row (tmp0/1 set before use) */
            for (uint64_t k = 0; k < n_ops && !bad; k++) {
                int na;
                if (parser == 4) {
                    na = op_52ns(&e, ops[k], args, ia, i, t3);
                } else {
                    na = op_common(&e, ops[k], args, ia, i, t1, t3);
                    if (na < 0) na = parser == 3 ? op_42ns(&e, ops[k], args, ia, i, t1, t3)
                                                 : op_stage3(&e, ops[k], args, ia, i, t1, t3);
                }
                if (na < 0) bad = -1;
                ia += (uint64_t)(na < 0 ? 0 : na);
                if (ia > n_args) bad = -1;
            }
            if (!bad && ia != n_args) bad = -1;
            if (!bad && e.err) bad = e.err == 1 ? -2 : e.err == 2 ? -3 : e.err == 5 ? -5 : -4;
        }
#pragma omp critical
        if (bad && !status) status = bad;
        free(t1);
        free(t3);
    }
    return status;
}

/* parser: 0 step2prev, 1 step3prev, 2 step3, 3 step42ns, 4 step52ns.
 * Returns 0, or -1 (unknown opcode / argument overrun), -2 (an access outside
 * the given sections), -3 (a shifted access whose modulus is not native_dom),
 * -4 (q_2ns store without an output). */
int oc_parser_eval(int parser, const uint64_t *ops, uint64_t n_ops, const uint64_t *args, uint64_t n_args,
                   uint32_t n_sec, const uint64_t *sec_off, const uint64_t *sec_stride, uint64_t *const *sec_ptr,
                   const uint64_t *cpols, uint64_t numpols, uint64_t dom, uint64_t native_dom, uint32_t n_tmp1,
                   uint32_t n_tmp3, const uint64_t *challenges, const uint64_t *publics, const uint64_t *evals,
                   const uint64_t *x, const uint64_t *zhinv, uint64_t zhinv_size, const uint64_t *xdiv,
                   const uint64_t *xdivw, uint64_t *q, uint64_t *f)
{
    return parser_run(parser, ops, n_ops, args, n_args, n_sec, sec_off, sec_stride, sec_ptr, cpols, numpols, dom,
                      native_dom, n_tmp1, n_tmp3, challenges, publics, evals, x, zhinv, zhinv_size, xdiv, xdivw, q, f,
                      NULL, 0, NULL, 0);
}

/* The same interpreter on sampled rows of a dom-row domain too large to hold
 * on the host: rows[0..n_rows) are evaluated (row indices of the whole
 * domain: shifts wrap mod dom, zhInv by the true row), and every row-indexed
 * input and output -- the sections, constant pols, x, xDivXSub, q / f --
 * holds only the rows rmap[0..nmap) (sorted ascending, every evaluated row and
 * every row a shifted access reaches), row r at its index in rmap.  Returns
 * as oc_parser_eval, or -5 (an access to a row missing from rmap). */
int oc_parser_eval_rows(int parser, const uint64_t *ops, uint64_t n_ops, const uint64_t *args, uint64_t n_args,
                        uint32_t n_sec, const uint64_t *sec_off, const uint64_t *sec_stride, uint64_t *const *sec_ptr,
                        const uint64_t *cpols, uint64_t numpols, uint64_t dom, uint64_t native_dom, uint32_t n_tmp1,
                        uint32_t n_tmp3, const uint64_t *challenges, const uint64_t *publics, const uint64_t *evals,
                        const uint64_t *x, const uint64_t *zhinv, uint64_t zhinv_size, const uint64_t *xdiv,
                        const uint64_t *xdivw, uint64_t *q, uint64_t *f, const uint64_t *rows, uint64_t n_rows,
                        const uint64_t *rmap, uint64_t nmap)
{
    for (uint64_t k = 1; k < nmap; k++)
        if (rmap[k] <= rmap[k - 1]) return -6; /* rmap must be strictly ascending */
    return parser_run(parser, ops, n_ops, args, n_args, n_sec, sec_off, sec_stride, sec_ptr, cpols, numpols, dom,
                      native_dom, n_tmp1, n_tmp3, challenges, publics, evals, x, zhinv, zhinv_size, xdiv, xdivw, q, f,
                      rows, n_rows, rmap, nmap);
}
