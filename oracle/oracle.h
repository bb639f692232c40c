/*
 * oracle/oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C + OpenMP) of the reference's STARK hot-path
 * primitives.  It is the checker for the HIP product path (tests/, smoke(),
 * bench.py's cpu_baseline leg) and never part of the product: nothing under
 * zkevm-prover_amd/ links or calls it.
 *
 * Pinning: tests/test_golden_proofs.py replays the reference's own golden
 * proofs (testvectors/aggregatedProof/recursive1.zkin.proof_0.json and
 * testvectors/finalProof/recursive2.zkin.proof_01.json, committed under
 * tests/golden/) through this library: transcript -> query indices, every
 * Merkle opening of every tree, every FRI fold and the last fold into finalPol.
 * The large NTT/LDE is pinned by the naive-DFT cross-check at small n plus the
 * golden FRI folds (16-point INTTs) -- see DESIGN.md "Oracle".
 *
 * All buffers are row-major u64, exactly like the reference boundary
 * (stark_info.cpp:473-482).  Extension-field elements are 3 consecutive u64.
 */
#ifndef ORACLE_H
#define ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- field (gl.h exposes the inline versions) ---- */
uint64_t oc_gl_mul(uint64_t a, uint64_t b);
uint64_t oc_gl_add(uint64_t a, uint64_t b);
uint64_t oc_gl_sub(uint64_t a, uint64_t b);
uint64_t oc_gl_inv(uint64_t a);
uint64_t oc_gl_pow(uint64_t a, uint64_t e);
uint64_t oc_gl_w(unsigned n);
void oc_gl3_mul(uint64_t *o, const uint64_t *a, const uint64_t *b);
void oc_powers3(uint64_t *out, const uint64_t *base, uint64_t n);
void oc_gl3_inv(uint64_t *o, const uint64_t *a);

/* ---- NTT family (ntt.c) ----
 * NTT_Goldilocks::NTT / INTT (starks.cpp:262,285,326-327; friProve.cpp:102):
 * per column, natural order in and out, omega_n = W[log2 n]; INTT scales 1/n.
 * dst may equal src. */
void oc_ntt(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols, int inverse);
/* O(n^2) definition, small n only (checker of the checker) */
void oc_dft_naive(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols, int inverse);
/* NTT_Goldilocks::extendPol (starks.cpp:53,134,215):
 * out[i][c] = P_c(shift * omega_{n_ext}^i), P_c interpolating in[.][c] on <omega_n>.
 * out must hold n_ext*ncols; in is not modified. */
void oc_extend_pol(uint64_t *out, const uint64_t *in, uint64_t n_ext, uint64_t n, uint64_t ncols);

/* ---- Poseidon-GL (poseidon.c) ---- */
void oc_poseidon_full(uint64_t out[12], const uint64_t in[12]);       /* hash_full_result */
void oc_poseidon_hash(uint64_t out[4], const uint64_t in[12]);        /* hash */
void oc_linear_hash(uint64_t out[4], const uint64_t *in, uint64_t size);

/* ---- Merkle tree GL (merkle.c) ---- */
uint64_t oc_merkle_num_elements(uint64_t nrows);
/* PoseidonGoldilocks::merkletree: nodes = leaves(4*nrows) ++ levels ... ++ root */
void oc_merkletree(uint64_t *nodes, const uint64_t *src, uint64_t ncols, uint64_t nrows);
void oc_merkle_root(uint64_t root[4], const uint64_t *nodes, uint64_t nrows);
uint64_t oc_merkle_proof_size(uint64_t nrows); /* number of sibling digests */
/* MerkleTreeGL::getGroupProof: proof = row values (ncols) ++ siblings (4 each) */
void oc_merkle_group_proof(uint64_t *proof, const uint64_t *nodes, const uint64_t *src,
                           uint64_t ncols, uint64_t nrows, uint64_t idx);
/* recompute the root from an opening; returns root in root_out */
void oc_merkle_root_from_proof(uint64_t root_out[4], const uint64_t *vals, uint64_t ncols,
                               const uint64_t *siblings, uint64_t nsiblings, uint64_t idx);

/* ---- Transcript (transcript.c) ---- */
typedef struct {
    uint64_t state[4];
    uint64_t pending[8];
    uint64_t out[12];
    uint32_t pending_cursor;
    uint32_t out_cursor;
} oc_transcript;
void oc_transcript_init(oc_transcript *t);
void oc_transcript_put(oc_transcript *t, const uint64_t *in, uint64_t n);
uint64_t oc_transcript_get_fields1(oc_transcript *t);
void oc_transcript_get_field(oc_transcript *t, uint64_t out[3]);
void oc_transcript_get_permutations(oc_transcript *t, uint64_t *res, uint64_t n, uint64_t nbits);

/* ---- FRI (fri.c) ----
 * One FRIProve::prove fold step (friProve.cpp:20-108) for si > 0:
 * pol has 2^pol_bits ext elements, out gets 2^out_bits ext elements.
 * shift_inv is polShiftInv for this step (7^-1 squared per reduced bit so far). */
void oc_fri_fold(uint64_t *out, const uint64_t *pol, uint64_t pol_bits, uint64_t out_bits,
                 const uint64_t special_x[3], uint64_t shift_inv);
/* fold of a single group (the values a query opens): vals = nx ext elements
 * pol[g + j*2^out_bits], j < nx */
void oc_fri_fold_group(uint64_t out[3], const uint64_t *vals, uint64_t nx, uint64_t g,
                       uint64_t pol_bits, const uint64_t special_x[3], uint64_t shift_inv);
/* FRIProve::getTransposed (friProve.cpp:252-270) on ext elements */
void oc_fri_get_transposed(uint64_t *aux, const uint64_t *pol, uint64_t degree, uint64_t transpose_bits);

/* ---- STARK stages (stark.c) ---- */
uint64_t oc_rand_u64(uint64_t seed, uint64_t stream, uint64_t col, uint64_t row);
void oc_rand_cols(uint64_t *buf, uint64_t stride, const uint32_t *cols, uint64_t ncols, uint64_t nrows, uint64_t seed,
                  uint64_t stream);
struct zxp_instr_s;
void oc_zxp_eval(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_tmp1, uint32_t n_tmp3,
                 uint64_t **sec, const uint64_t *stride, uint64_t dom, const uint64_t *challenges,
                 const uint64_t *publics, const uint64_t *evals, const uint64_t *x, const uint64_t *xdiv,
                 const uint64_t *xdivw, const uint64_t *zhinv, uint64_t zhinv_size);
void oc_zxc_eval(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_tmp1, uint32_t n_tmp3,
                 const void *term, const uint64_t *cst, uint64_t **sec, const uint64_t *stride, uint64_t dom,
                 const uint64_t *challenges, const uint64_t *publics, const uint64_t *evals, const uint64_t *x,
                 const uint64_t *xdiv, const uint64_t *xdivw, const uint64_t *zhinv, uint64_t zhinv_size);
int oc_calculate_z(uint64_t *z, uint64_t zs, const uint64_t *num, uint64_t ns, const uint64_t *den, uint64_t ds,
                   uint64_t n);
void oc_evmap(uint64_t *evals, const uint64_t *const *pols, const uint64_t *strides, const uint32_t *dims,
              const uint32_t *primes, uint64_t n_ev, const uint64_t *lev, const uint64_t *lpev, uint64_t n,
              uint32_t extend_bits);
void oc_xdivxsub(uint64_t *xdiv, uint64_t *xdivw, const uint64_t *x, uint64_t n, const uint64_t xi[3], uint64_t w);
void oc_powers(uint64_t *out, uint64_t start, uint64_t w, uint64_t n);

/* ---- misc ---- */
void oc_batch_inverse3(uint64_t *out, const uint64_t *in, uint64_t n); /* Polinomial::batchInverse */
/* ---- plookup h1/h2 (h1h2.c): returns 0, or 1 + first f row not in t ---- */
uint64_t oc_h1h2(uint64_t *h1, uint64_t h1s, uint64_t *h2, uint64_t h2s, const uint64_t *f, uint64_t fs,
                 const uint64_t *t, uint64_t ts, uint64_t n, uint32_t dim);
int oc_num_threads(void);
void oc_set_num_threads(int n);

#ifdef __cplusplus
}
#endif
#endif /* ORACLE_H */
