/*
 * oracle/stark.c -- TEST INFRASTRUCTURE ONLY (CPU oracle of the STARK stages).
 *
 *  - oc_zxp_eval: the expression programs (include/zkgpu_zxp.h), i.e. the role
 *    of Steps::step2prev/step3prev/step42ns/step52ns (steps.hpp:21-58); op
 *    semantics as the reference's generated code / bytecode tables
 *    (e.g. recursive1.chelpers.step42ns.cpp, zkevm.chelpers.step42ns.parser.cpp:24-784,
 *    step52ns.parser.cpp:9-226): base/ext add, sub, mul, copy; x_n / x_2ns;
 *    zhInv (zhInv.cpp:7-31); xDivXSubXi / xDivXSubWXi; challenges; evals.
 *  - oc_calculate_z: Polinomial::calculateZ (polinomial.hpp:586-607).
 *  - oc_evmap: Starks::evmap (starks.cpp:556-669).
 *  - oc_xdivxsub: starks.cpp:344-366.
 * Sections are row-major (row stride = section width), like the reference's
 * memory map (stark_info.cpp:473-482).
 */
#include <stdlib.h>
#include <string.h>
#include <omp.h>
#include "gl.h"
#include "oracle.h"
#include "../include/zkgpu_zxp.h"

uint64_t oc_rand_u64(uint64_t seed, uint64_t stream, uint64_t col, uint64_t row)
{
    uint64_t x = seed ^ (stream << 56) ^ (col * 0x9E3779B97F4A7C15ULL) ^ (row * 0xC2B2AE3D27D4EB4FULL);
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return z >> 1;
}

void oc_rand_cols(uint64_t *buf, uint64_t stride, const uint32_t *cols, uint64_t ncols, uint64_t nrows, uint64_t seed,
                  uint64_t stream)
{
#pragma omp parallel for schedule(static)
    for (uint64_t r = 0; r < nrows; r++)
        for (uint64_t k = 0; k < ncols; k++) buf[r * stride + cols[k]] = oc_rand_u64(seed, stream, cols[k], r);
}

typedef struct {
    uint64_t v[3];
    int dim;
} val;

typedef struct {
    uint64_t **sec;       /* SEC_COUNT row-major section bases */
    const uint64_t *stride; /* row stride per section */
    uint64_t dom;         /* rows of the evaluation domain */
    const uint64_t *challenges, *publics, *evals;
    const uint64_t *x;    /* x_i of the domain (dom entries) */
    const uint64_t *xdiv, *xdivw; /* dom x 3 (2n domain only) */
    const uint64_t *zhinv; /* 2^eb entries */
    uint64_t zhinv_mask;
    const uint64_t *cst;   /* compiled programs: ZXP_IMM constants (3 each) */
    const zxp_term *term;  /* compiled programs: DOT terms */
} env_t;

static inline val load(const env_t *e, const zxp_operand *o, const uint64_t *t1, const uint64_t *t3, uint64_t i)
{
    val r = {{0, 0, 0}, 1};
    switch (o->kind) {
    case ZXP_TMP1: r.v[0] = t1[o->a]; break;
    case ZXP_TMP3: memcpy(r.v, t3 + 3 * o->a, 24); r.dim = 3; break;
    case ZXP_COL:
    case ZXP_COL3: {
        uint64_t row = (i + (uint64_t)(int64_t)(int32_t)o->c + e->dom) % e->dom;
        const uint64_t *p = e->sec[o->a] + row * e->stride[o->a] + o->b;
        r.v[0] = p[0];
        if (o->kind == ZXP_COL3) {
            r.v[1] = p[1];
            r.v[2] = p[2];
            r.dim = 3;
        }
        break;
    }
    case ZXP_LIT: r.v[0] = (uint64_t)o->a | ((uint64_t)o->b << 32); break;
    case ZXP_CHAL: memcpy(r.v, e->challenges + 3 * o->a, 24); r.dim = 3; break;
    case ZXP_PUB: r.v[0] = e->publics[o->a]; break;
    case ZXP_X: r.v[0] = e->x[i]; break;
    case ZXP_EVAL: memcpy(r.v, e->evals + 3 * o->a, 24); r.dim = 3; break;
    case ZXP_XDIV: memcpy(r.v, e->xdiv + 3 * i, 24); r.dim = 3; break;
    case ZXP_XDIVW: memcpy(r.v, e->xdivw + 3 * i, 24); r.dim = 3; break;
    case ZXP_ZI: r.v[0] = e->zhinv[i & e->zhinv_mask]; break;
    case ZXP_IMM: memcpy(r.v, e->cst + 3 * o->a, 24); r.dim = (int)o->b; break;
    default: break;
    }
    return r;
}

/* compiled DOT (include/zkgpu_zxp.h): sum of coef * (base source value) */
static inline val dot(const env_t *e, const zxp_operand *opnd, const zxp_instr *in, const uint64_t *t1,
                      const uint64_t *t3, uint64_t i)
{
    val r = {{0, 0, 0}, in->op == ZXP_DOT3 ? 3 : 1};
    for (uint32_t k = in->a; k < in->a + in->b; k++) {
        const zxp_term *t = &e->term[k];
        uint64_t x = 1;
        if (t->src != ZXP_TERM_ONE) {
            val s = load(e, &opnd[t->src], t1, t3, i);
            x = s.v[t->comp];
        }
        for (int c = 0; c < 3; c++) r.v[c] = gl_add(r.v[c], gl_mul(t->coef[c], x));
    }
    return r;
}

static inline void store(const env_t *e, const zxp_operand *o, uint64_t *t1, uint64_t *t3, uint64_t i, const val *v)
{
    switch (o->kind) {
    case ZXP_TMP1: t1[o->a] = v->v[0]; break;
    case ZXP_TMP3:
        t3[3 * o->a] = v->v[0];
        t3[3 * o->a + 1] = v->dim == 3 ? v->v[1] : 0;
        t3[3 * o->a + 2] = v->dim == 3 ? v->v[2] : 0;
        break;
    case ZXP_COL:
    case ZXP_COL3: {
        /* a shifted store writes row (i + shift) mod dom (parser opcodes 101-114, 119) */
        const uint64_t row = (i + (uint64_t)(int64_t)(int32_t)o->c + e->dom) % e->dom;
        uint64_t *p = e->sec[o->a] + row * e->stride[o->a] + o->b;
        p[0] = gl_canon(v->v[0]);
        if (o->kind == ZXP_COL3) {
            p[1] = v->dim == 3 ? gl_canon(v->v[1]) : 0;
            p[2] = v->dim == 3 ? gl_canon(v->v[2]) : 0;
        }
        break;
    }
    default: break;
    }
}

static inline val binop(uint32_t op, const val *a, const val *b)
{
    val r;
    r.dim = (a->dim == 3 || b->dim == 3) ? 3 : 1;
    if (op == ZXP_MUL) {
        if (a->dim == 3 && b->dim == 3) {
            gl3_mul(r.v, a->v, b->v);
        } else if (a->dim == 3) {
            gl3_mul1(r.v, a->v, b->v[0]);
        } else if (b->dim == 3) {
            gl3_mul1(r.v, b->v, a->v[0]);
        } else {
            r.v[0] = gl_mul(a->v[0], b->v[0]);
            r.v[1] = r.v[2] = 0;
        }
        return r;
    }
    /* add / sub: a base operand contributes to component 0 only */
    uint64_t av[3] = {a->v[0], a->dim == 3 ? a->v[1] : 0, a->dim == 3 ? a->v[2] : 0};
    uint64_t bv[3] = {b->v[0], b->dim == 3 ? b->v[1] : 0, b->dim == 3 ? b->v[2] : 0};
    for (int k = 0; k < 3; k++) r.v[k] = op == ZXP_ADD ? gl_add(av[k], bv[k]) : gl_sub(av[k], bv[k]);
    return r;
}

static void zxp_run(const void *instr_v, uint32_t n_instr, const void *opnd_v, uint32_t n_tmp1, uint32_t n_tmp3,
                    uint64_t **sec, const uint64_t *stride, uint64_t dom, const uint64_t *challenges,
                    const uint64_t *publics, const uint64_t *evals, const uint64_t *x, const uint64_t *xdiv,
                    const uint64_t *xdivw, const uint64_t *zhinv, uint64_t zhinv_size, const uint64_t *cst,
                    const zxp_term *term)
{
    const zxp_instr *instr = (const zxp_instr *)instr_v;
    const zxp_operand *opnd = (const zxp_operand *)opnd_v;
    env_t e = {sec, stride, dom, challenges, publics, evals, x, xdiv, xdivw, zhinv, zhinv_size ? zhinv_size - 1 : 0,
               cst, term};
#pragma omp parallel
    {
        uint64_t *t1 = (uint64_t *)calloc(n_tmp1 + 1, sizeof(uint64_t));
        uint64_t *t3 = (uint64_t *)calloc(3 * n_tmp3 + 3, sizeof(uint64_t));
#pragma omp for schedule(static)
        for (uint64_t i = 0; i < dom; i++) {
            /* every row starts with zero temporaries (the compiled programs'
             * convention; the reference's step52ns zeroes tmp2 per row) */
            memset(t1, 0, (n_tmp1 + 1) * sizeof(uint64_t));
            memset(t3, 0, (3 * n_tmp3 + 3) * sizeof(uint64_t));
            for (uint32_t k = 0; k < n_instr; k++) {
                const zxp_instr *in = &instr[k];
                val a = {{0, 0, 0}, 1};
                if (in->op <= ZXP_COPY) a = load(&e, &opnd[in->a], t1, t3, i);
                val r;
                if (in->op == ZXP_DOT1 || in->op == ZXP_DOT3) {
                    r = dot(&e, opnd, in, t1, t3, i);
                } else if (in->op == ZXP_COPY) {
                    r = a;
                } else {
                    val b = load(&e, &opnd[in->b], t1, t3, i);
                    r = binop(in->op, &a, &b);
                }
                store(&e, &opnd[in->dst], t1, t3, i, &r);
            }
        }
        free(t1);
        free(t3);
    }
}

void oc_zxp_eval(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_tmp1, uint32_t n_tmp3,
                 uint64_t **sec, const uint64_t *stride, uint64_t dom, const uint64_t *challenges,
                 const uint64_t *publics, const uint64_t *evals, const uint64_t *x, const uint64_t *xdiv,
                 const uint64_t *xdivw, const uint64_t *zhinv, uint64_t zhinv_size)
{
    zxp_run(instr, n_instr, opnd, n_tmp1, n_tmp3, sec, stride, dom, challenges, publics, evals, x, xdiv, xdivw, zhinv,
            zhinv_size, NULL, NULL);
}

/* a compiled program (zkgpu_zxp_compile output): checks the compiler against
 * the source program on the same inputs */
void oc_zxc_eval(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_tmp1, uint32_t n_tmp3,
                 const void *term, const uint64_t *cst, uint64_t **sec, const uint64_t *stride, uint64_t dom,
                 const uint64_t *challenges, const uint64_t *publics, const uint64_t *evals, const uint64_t *x,
                 const uint64_t *xdiv, const uint64_t *xdivw, const uint64_t *zhinv, uint64_t zhinv_size)
{
    zxp_run(instr, n_instr, opnd, n_tmp1, n_tmp3, sec, stride, dom, challenges, publics, evals, x, xdiv, xdivw, zhinv,
            zhinv_size, cst, (const zxp_term *)term);
}

/* Polinomial::calculateZ: z[0] = 1, z[i] = z[i-1] * num[i-1] / den[i-1];
 * returns 1 if the product closes (z[n-1]*num[n-1]/den[n-1] == 1).
 * num/den/z are ext columns with row strides (in u64). */
int oc_calculate_z(uint64_t *z, uint64_t zs, const uint64_t *num, uint64_t ns, const uint64_t *den, uint64_t ds,
                   uint64_t n)
{
    uint64_t *d = (uint64_t *)malloc(sizeof(uint64_t) * 3 * n);
    uint64_t *di = (uint64_t *)malloc(sizeof(uint64_t) * 3 * n);
    for (uint64_t i = 0; i < n; i++) memcpy(d + 3 * i, den + i * ds, 24);
    oc_batch_inverse3(di, d, n);
    z[0] = 1;
    z[1] = 0;
    z[2] = 0;
    for (uint64_t i = 1; i < n; i++) {
        uint64_t t[3];
        gl3_mul(t, num + (i - 1) * ns, di + 3 * (i - 1));
        gl3_mul(z + i * zs, z + (i - 1) * zs, t);
    }
    uint64_t t[3], chk[3];
    gl3_mul(t, num + (n - 1) * ns, di + 3 * (n - 1));
    gl3_mul(chk, z + (n - 1) * zs, t);
    free(d);
    free(di);
    return chk[0] == 1 && chk[1] == 0 && chk[2] == 0;
}

/* Starks::evmap: evals[e] = sum_{k<N} L(k) * pol_e[k << extendBits] with
 * L = LEv or LpEv (N x 3).  pol pointers/strides/dims/primes per entry. */
void oc_evmap(uint64_t *evals, const uint64_t *const *pols, const uint64_t *strides, const uint32_t *dims,
              const uint32_t *primes, uint64_t n_ev, const uint64_t *lev, const uint64_t *lpev, uint64_t n,
              uint32_t extend_bits)
{
#pragma omp parallel for schedule(dynamic, 1)
    for (uint64_t e = 0; e < n_ev; e++) {
        uint64_t acc[3] = {0, 0, 0};
        const uint64_t *L = primes[e] ? lpev : lev;
        for (uint64_t k = 0; k < n; k++) {
            const uint64_t *p = pols[e] + (k << extend_bits) * strides[e];
            uint64_t t[3];
            if (dims[e] == 1)
                gl3_mul1(t, L + 3 * k, p[0]);
            else
                gl3_mul(t, L + 3 * k, p);
            gl3_add(acc, acc, t);
        }
        memcpy(evals + 3 * e, acc, 24);
    }
}

/* xDivXSubXi[k] = x_k / (x_k - xi), xDivXSubWXi[k] = x_k / (x_k - w xi),
 * x_k = 7 * w_{2n}^k (starks.cpp:344-366) */
void oc_xdivxsub(uint64_t *xdiv, uint64_t *xdivw, const uint64_t *x, uint64_t n, const uint64_t xi[3], uint64_t w)
{
    uint64_t wxi[3];
    gl3_mul1(wxi, xi, w);
    for (uint64_t k = 0; k < n; k++) {
        uint64_t xv[3] = {x[k], 0, 0};
        gl3_sub(xdiv + 3 * k, xv, xi);
        gl3_sub(xdivw + 3 * k, xv, wxi);
    }
    oc_batch_inverse3(xdiv, xdiv, n);
    oc_batch_inverse3(xdivw, xdivw, n);
#pragma omp parallel for schedule(static)
    for (uint64_t k = 0; k < n; k++) {
        gl3_mul1(xdiv + 3 * k, xdiv + 3 * k, x[k]);
        gl3_mul1(xdivw + 3 * k, xdivw + 3 * k, x[k]);
    }
}

/* x_i = start * w^i for i < n */
void oc_powers(uint64_t *out, uint64_t start, uint64_t w, uint64_t n)
{
#pragma omp parallel for schedule(static)
    for (uint64_t c = 0; c < n; c += 4096) {
        uint64_t v = gl_mul(start, gl_pow(w, c));
        uint64_t end = c + 4096 < n ? c + 4096 : n;
        for (uint64_t i = c; i < end; i++) {
            out[i] = v;
            v = gl_mul(v, w);
        }
    }
}
