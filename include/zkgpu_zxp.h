/*
 * zkgpu_zxp.h -- expression-program format ("ZXP") consumed by the STARK
 * expression evaluators (the role of the reference's Steps::step*_parser /
 * step*_first evaluators, steps.hpp:21-58; bytecode semantics per
 * zkevm.chelpers.step42ns.parser.cpp:24-784 and step52ns.parser.cpp:9-226).
 *
 * A program is a flat list of instructions evaluated once per row i of its
 * domain (n = 2^nBits for stage 2/3 programs, 2n = 2^nBitsExt for the
 * quotient and FRI programs).  Each instruction combines two operands and
 * writes a third:  dst = a (op) b.  Operand dimension is 1 (F_p) or 3 (F_p^3);
 * the result dimension is the larger one (F_p^3 x F_p = componentwise).
 *
 * Operand kinds (zxp_operand.kind):
 *   ZXP_TMP1  a = temp slot           (per-row base temporary)
 *   ZXP_TMP3  a = temp slot           (per-row extension temporary)
 *   ZXP_COL   a = section, b = column, c = row shift (int32)  -> base value
 *             pols[section][col][(i + shift) mod dom]
 *   ZXP_COL3  as ZXP_COL, columns b, b+1, b+2 form one F_p^3 value
 *   ZXP_LIT   a | b << 32  literal
 *   ZXP_CHAL  a = challenge index (F_p^3)
 *   ZXP_PUB   a = public input index
 *   ZXP_X     x_i of the domain: omega_n^i (n) or 7*omega_2n^i (2n)
 *   ZXP_EVAL  a = evals index (F_p^3)
 *   ZXP_XDIV  x_i/(x_i - xi)        (2n domain, F_p^3)
 *   ZXP_XDIVW x_i/(x_i - omega*xi)  (2n domain, F_p^3)
 *   ZXP_ZI    1/Z_H(x_i) (2n domain), zhInv.cpp:7-31
 * Instruction ops: ZXP_ADD, ZXP_SUB, ZXP_MUL, ZXP_COPY (dst = a).
 * A COL/COL3 destination writes the column (shift must be 0).
 */
#ifndef ZKGPU_ZXP_H
#define ZKGPU_ZXP_H
#include <stdint.h>

enum {
    ZXP_TMP1 = 0,
    ZXP_TMP3 = 1,
    ZXP_COL = 2,
    ZXP_COL3 = 3,
    ZXP_LIT = 4,
    ZXP_CHAL = 5,
    ZXP_PUB = 6,
    ZXP_X = 7,
    ZXP_EVAL = 8,
    ZXP_XDIV = 9,
    ZXP_XDIVW = 10,
    ZXP_ZI = 11
};
enum { ZXP_ADD = 0, ZXP_SUB = 1, ZXP_MUL = 2, ZXP_COPY = 3 };

/* STARK sections (the reference's eSection, stark_info.hpp) */
enum {
    SEC_CM1_N = 0,
    SEC_CM2_N = 1,
    SEC_CM3_N = 2,
    SEC_TMP_N = 3, /* tmpExp_n */
    SEC_CONST_N = 4,
    SEC_CM1_2NS = 5,
    SEC_CM2_2NS = 6,
    SEC_CM3_2NS = 7,
    SEC_CM4_2NS = 8,
    SEC_CONST_2NS = 9,
    SEC_Q_2NS = 10,
    SEC_F_2NS = 11,
    SEC_COUNT = 12
};

typedef struct {
    uint32_t kind, a, b, c;
} zxp_operand;

typedef struct {
    uint32_t op, dst, a, b;
} zxp_instr;

/* ---- compiled programs (zkgpu_zxp_compile, include/zkgpu.h) ---------------
 * The device does not interpret the producer's op list directly: the host
 * compiles it first.  Every value is tracked as an affine form
 * cst + sum_t coef_t * src_t over base-field row values src_t (columns, temps)
 * with row-constant F_p^3 coefficients (challenges, evals, publics, literals
 * and their products).  Additions, subtractions, copies and products by a
 * row-constant operand fold into the form on the host; a form is emitted as
 * ONE linear-combination instruction only where a row-varying product, a
 * column store or the term cap needs its value.  Horner chains such as the
 * reference's FRI polynomial (step52ns: acc = acc*v1 + pol_k) and constraint
 * combination (step42ns: acc = acc*alpha + C_k) become dot products with
 * precomputed challenge powers.  Field arithmetic is exact, so the compiled
 * program computes the same values as the source program.
 * Compiled instruction ops add:
 *   ZXP_DOT1 / ZXP_DOT3  dst = sum over terms [a, a+b) of coef * src
 *                        (result dimension 1 / 3)
 * and operand kinds add:
 *   ZXP_IMM   a = index into the constant table (3 u64 per entry), b = dim.
 * Temporaries are SSA values packed into slots (liveness linear scan). */
enum { ZXP_DOT1 = 4, ZXP_DOT3 = 5 };
enum { ZXP_IMM = 12 };
#define ZXP_TERM_ONE 0xFFFFFFFFu /* term source "1": the form's constant */

typedef struct {
    uint32_t src;  /* operand index (COL / TMP1 / TMP3) or ZXP_TERM_ONE */
    uint32_t comp; /* component of a TMP3 source */
    uint64_t coef[3];
} zxp_term;

typedef struct {
    const zxp_instr *instr;
    uint32_t n_instr;
    const zxp_operand *opnd;
    uint32_t n_opnd;
    const zxp_term *term;
    uint32_t n_term;
    const uint64_t *cst; /* n_cst x 3 */
    uint32_t n_cst;
    uint32_t n_tmp1, n_tmp3;
} zxp_compiled;

typedef struct {
    const zxp_instr *instr;
    uint32_t n_instr;
    const zxp_operand *opnd;
    uint32_t n_opnd;
    uint32_t n_tmp1, n_tmp3; /* temp slots */
    uint32_t domain_ext;     /* 0: n-domain, 1: 2n-domain */
} zxp_program;

#endif /* ZKGPU_ZXP_H */
