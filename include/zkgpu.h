/*
 * zkgpu.h -- C-ABI of libzkgpu, the MI355X (gfx950) STARK hot path for
 * zkevm-prover.  Plain pointers and sizes only; every function returns
 * ZKGPU_OK (0) or a negative error code, details in zkgpu_last_error().
 *
 * Two families:
 *   - host-pointer drop-ins with the reference's row-major buffers
 *     (stark_info.cpp:473-482 layout).  The library stages H2D, runs the HIP
 *     kernels on its device copy (column-major "SoA" internally), and copies
 *     the result back.  These are what the reference's C++ call sites bind to
 *     (see INTEGRATION.md for the adapter classes).
 *   - *_dev functions on device-resident column-major buffers (column c at
 *     ptr + c*ld), for traces kept in HBM across stages.  No host copies.
 *
 * Element type: Goldilocks u64, p = 2^64 - 2^32 + 1; inputs may be
 * non-canonical, outputs are canonical.  Extension elements are 3 u64.
 *
 * Threading: one calling host thread per process/device (the reference calls
 * genProof from one thread, prover.cpp:182-255).  Kernels are enqueued on
 * the stream given to zkgpu_set_stream (default: the null stream); host-
 * pointer calls synchronise that stream before returning, *_dev calls do not.
 */
#ifndef ZKGPU_H
#define ZKGPU_H

#include <stdint.h>
#include "zkgpu_zxp.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ZKGPU_OK 0
#define ZKGPU_ERR_HIP -1   /* HIP runtime error */
#define ZKGPU_ERR_ARG -2   /* invalid argument / unsupported size */
#define ZKGPU_ERR_INIT -3  /* zkgpu_init not called or failed */
#define ZKGPU_ERR_OOM -4   /* device allocation failed */

/* ---- lifecycle ------------------------------------------------------------
 * Replaces the implicit setup of the Goldilocks submodule objects:
 * NTT_Goldilocks(maxDomainSize, nThreads, extension) constructed at
 * starks.hpp:81-82 and friProve.cpp:100 (twiddle tables), plus the Poseidon
 * constant tables.  device = HIP device ordinal; device < 0 keeps the
 * initialised device, or uses the calling thread's current HIP device. */
int zkgpu_init(int device);
void zkgpu_release(void);
const char *zkgpu_last_error(void);
int zkgpu_set_stream(void *hip_stream);
/* the stream every zkgpu call is enqueued on (collectives of a sharded
 * prover are enqueued on it too, include/zkgpu_stark.h zkgpu_comm) */
void *zkgpu_get_stream(void);
int zkgpu_synchronize(void);
/* number of exported entry points (ABI self-check for tests) */
int zkgpu_abi_version(void);

/* ---- NTT ---------------------------------------------------------------
 * NTT_Goldilocks::NTT / INTT(Element *dst, Element *src, uint64_t size,
 * uint64_t ncols, Element *buffer, uint64_t nphase, uint64_t nblock)
 * -- starks.cpp:262 (INTT NE x 3), :285 (NTT NE x 6), :326-327 (INTT N x 3),
 * friProve.cpp:102.  Row-major n x ncols, natural order; INTT scales 1/n.
 * dst may equal src.  n must be a power of two <= 2^28. */
int zkgpu_gl_ntt(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols, int inverse);

/* NTT_Goldilocks::extendPol(Element *output, Element *input, uint64_t N_Extended,
 * uint64_t N, uint64_t ncols, Element *buffer) -- starks.cpp:53,134,215.
 * out[i][c] = P_c(7 * omega_{n_ext}^i), P_c interpolating in[.][c] on <omega_n>.
 * Row-major in (n x ncols) and out (n_ext x ncols). */
int zkgpu_gl_extend_pol(uint64_t *out, const uint64_t *in, uint64_t n_ext, uint64_t n, uint64_t ncols);

/* device bytes extend_pol keeps in its grow-only workspaces for ncols
 * columns (column batches; for the host's memory plan, no GPU needed) */
uint64_t zkgpu_lde_workspace_bytes(uint64_t n, uint64_t n_ext, uint64_t ncols);
/* at most max_cols columns per extend_pol batch (0: the default, 2^31 words
 * of n_ext-row scratch): a smaller batch bounds the LDE workspace (and, in the
 * tests, exercises the column batching at small sizes).  Process-wide. */
void zkgpu_set_lde_batch_cols(uint64_t max_cols);

/* device-resident, column-major variants */
int zkgpu_gl_ntt_dev(uint64_t *dst, uint64_t ld_dst, const uint64_t *src, uint64_t ld_src, uint64_t n,
                     uint64_t ncols, int inverse);
int zkgpu_gl_extend_pol_dev(uint64_t *out, uint64_t ld_out, const uint64_t *in, uint64_t ld_in, uint64_t n_ext,
                            uint64_t n, uint64_t ncols);
/* extendPol in place (the same transform, starks.cpp:53,215): base holds
 * ncols n-row columns packed at ld n on entry and the ncols n_ext-row columns
 * at ld n_ext on return (base must hold ncols * n_ext words).  Column batches
 * run from the last down, each read whole into the LDE workspace before its
 * output is stored, so no column is overwritten before it is read; lets a
 * prover extend a section into the memory its n-domain values occupied
 * (host/starks.cpp, the lean memory plan).  Same values as extendPol
 * (starks.cpp:53,134,215) out of place. */
int zkgpu_gl_extend_pol_inplace_dev(uint64_t *base, uint64_t n_ext, uint64_t n, uint64_t ncols);
/* row-major <-> column-major on device (boundary layout change) */
int zkgpu_rows_to_cols_dev(uint64_t *cols, uint64_t ld, const uint64_t *rows, uint64_t nrows, uint64_t ncols);
int zkgpu_cols_to_rows_dev(uint64_t *rows, const uint64_t *cols, uint64_t ld, uint64_t nrows, uint64_t ncols);

/* ---- Poseidon-GL --------------------------------------------------------
 * PoseidonGoldilocks::hash_full_result(Element out[12], const Element in[12])
 * -- transcript.cpp:23,46.  Computed on the GPU. */
int zkgpu_gl_poseidon_full(uint64_t out[12], const uint64_t in[12]);
/* The same permutation on the host CPU (no GPU, no zkgpu_init): the
 * transcript's (Transcript::put/getFields, transcript.cpp:18-24 ->
 * PoseidonGoldilocks::hash_full_result), where one serial permutation sits on
 * the critical path and a GPU launch would only add latency. */
int zkgpu_gl_poseidon_full_host(uint64_t out[12], const uint64_t in[12]);
/* PoseidonGoldilocks::hash(Element out[4], const Element in[12]) */
int zkgpu_gl_poseidon_hash(uint64_t out[4], const uint64_t in[12]);
/* PoseidonGoldilocks::linear_hash(Element *out, Element *in, uint64_t size)
 * -- main_sm/fork_9/main_exec (utils.cpp:708).  One input row. */
int zkgpu_gl_linear_hash(uint64_t out[4], const uint64_t *in, uint64_t size);
/* batched permutation on device: in/out are n x 12 (full) or out n x 4 */
int zkgpu_gl_poseidon_batch_dev(uint64_t *out, const uint64_t *in, uint64_t n, int full);

/* ---- Merkle tree GL ----------------------------------------------------
 * MerklehashGoldilocks::getTreeNumElements(nrows) (stark_info.hpp:332,
 * build_const_tree.cpp:566-569): 4*nrows + 4*(nrows-1). */
uint64_t zkgpu_gl_merkle_num_elements(uint64_t nrows);
/* PoseidonGoldilocks::merkletree{,_avx,_avx512}(Element *tree, Element *input,
 * uint64_t ncols, uint64_t nrows) -- merkleTreeGL.cpp:37-44,
 * build_const_tree.cpp:582.  Row-major source; nrows a power of two. */
int zkgpu_gl_merkletree(uint64_t *nodes, const uint64_t *src, uint64_t ncols, uint64_t nrows);
/* device-resident: src column-major (ld), nodes on device */
int zkgpu_gl_merkletree_dev(uint64_t *nodes, const uint64_t *src, uint64_t ld, uint64_t ncols, uint64_t nrows);
/* the same tree over a section held in two regions: columns [0, split) at
 * src + c*ld, columns [split, ncols) at src2 + (c - split)*ld (split a
 * multiple of 8: the linear hash absorbs 8 columns at a time).  The lean
 * memory plan's stage-1 commit (host/starks.cpp); same nodes as the
 * reference's merkelize of the whole section (merkleTreeGL.cpp:37-44). */
int zkgpu_gl_merkletree2_dev(uint64_t *nodes, const uint64_t *src, const uint64_t *src2, uint64_t ld, uint64_t split,
                             uint64_t ncols, uint64_t nrows);
/* device-resident, row-major source (FRI trees: friProve.cpp:117-121) */
int zkgpu_gl_merkletree_rows_dev(uint64_t *nodes, const uint64_t *src, uint64_t ncols, uint64_t nrows);
/* ---- constant tree (tools/starkpil/bctree) -----------------------------
 * Element count of a const-tree file: header 2 + nPols*nExt + tree
 * (build_const_tree.cpp:566-569). */
uint64_t zkgpu_const_tree_num_elements(uint64_t n_pols, uint32_t n_bits_ext);
/* build_const_tree.cpp:553-603 (GL hash): interpolate (extendPol of the
 * row-major N x nPols constant pols to nExt rows) + PoseidonGoldilocks::
 * merkletree, written in the file layout [nPols, nExt, LDE row-major,
 * tree nodes]; the verkey constRoot is the last 4 elements.  Host pointers. */
int zkgpu_build_const_tree(uint64_t *tree_out, const uint64_t *const_pols, uint64_t n_pols, uint32_t n_bits,
                           uint32_t n_bits_ext);

/* ---- executor hand-off ------------------------------------------------
 * Load a host row-major section (the committed-pols buffer the executor
 * fills, CommitPols stride = width, commit_pols.hpp:18,1735-1737; read by
 * prover.cpp:94-116) into device column-major storage (column c at
 * cols + c*ld), streamed in row blocks: each block's H2D copy runs on a copy
 * stream while the previous block is transposed, so a pinned (registered)
 * source moves at link speed.  register_host = 1 page-locks `rows` for the
 * duration of the call (hipHostRegister). */
int zkgpu_load_rows_dev(uint64_t *cols, uint64_t ld, const uint64_t *rows, uint64_t nrows, uint64_t ncols,
                        uint64_t block_rows, int register_host);
/* The same load in the background: a host thread of the library runs the
 * block loop on streams of its own (stage: caller-owned device buffer of at
 * least zkgpu_load_rows_stage_bytes bytes), so kernels on the library stream
 * -- the previous proof -- run while the trace crosses PCIe.  `rows`, `cols`
 * and `stage` stay untouched by the caller until zkgpu_load_wait(ticket)
 * returns (the load's status, and on failure the loader's message in
 * zkgpu_last_error() of the waiting thread; the ticket is freed).  The load
 * is ordered after everything already queued on the library stream (e.g. the
 * zeroing of freshly allocated `cols` / `stage`).  No reference
 * counterpart: the reference's batch prover loads each trace before its
 * genProof (prover.cpp:94-116). */
uint64_t zkgpu_load_rows_stage_bytes(uint64_t nrows, uint64_t ncols, uint64_t block_rows);
int zkgpu_load_rows_async(uint64_t *cols, uint64_t ld, const uint64_t *rows, uint64_t nrows, uint64_t ncols,
                          uint64_t block_rows, uint64_t *stage, uint64_t stage_bytes, void **ticket);
int zkgpu_load_wait(void *ticket);

/* MerkleTreeGL::getGroupProof(Element *proof, uint64_t idx) for nq queries at
 * once -- merkleTreeGL.cpp:12-35, friProve.cpp:195-232.
 * vals_out: nq x ncols, sibs_out: nq x log2(nrows) x 4 (host pointers);
 * src column-major on device (ld), nodes on device. */
int zkgpu_gl_merkle_open_dev(uint64_t *vals_out, uint64_t *sibs_out, const uint64_t *nodes, const uint64_t *src,
                             uint64_t ld, uint64_t ncols, uint64_t nrows, const uint64_t *idx, uint64_t nq);

/* ---- FRI -----------------------------------------------------------------
 * One fold step of FRIProve::prove (friProve.cpp:20-108), device-resident:
 * pol has 2^pol_bits ext elements (interleaved, 3 u64 each), out 2^out_bits.
 * special_x: host pointer to 3 u64; shift_inv: polShiftInv of this step. */
int zkgpu_fri_fold_dev(uint64_t *out, const uint64_t *pol, uint32_t pol_bits, uint32_t out_bits,
                       const uint64_t special_x[3], uint64_t shift_inv);
/* The same fold for output groups [g0, g0 + ngroups) only, reading those
 * groups' getTransposed rows (row g - g0 = the 2^(pol_bits - out_bits)
 * elements pol[g + i 2^out_bits], 3 u64 each: the layout
 * zkgpu_fri_transpose_dev writes with transpose_bits = out_bits); out gets
 * the ngroups folded elements.  The row-sharded prover's first fold, each
 * rank on its block of groups (friProve.cpp:44-108 restricted to g). */
int zkgpu_fri_fold_rows_dev(uint64_t *out, const uint64_t *rows, uint64_t g0, uint64_t ngroups, uint32_t pol_bits,
                            uint32_t out_bits, const uint64_t special_x[3], uint64_t shift_inv);
/* FRIProve::getTransposed (friProve.cpp:252-270), ext elements, device */
int zkgpu_fri_transpose_dev(uint64_t *aux, const uint64_t *pol, uint64_t degree, uint32_t transpose_bits);

/* ---- calculateH1H2 over row-sharded f / t --------------------------------
 * Polinomial::calculateH1H2_opt1/opt3 (polinomial.hpp:349-583, starks.cpp:
 * 104-127) when W ranks each hold rows [row0, row0 + nrows) of f and t (the
 * row-sharded prover, host/sharded_starks.hpp; the same h1 / h2 as
 * zkgpu_h1h2_dev on the whole columns).  Records are 5 u64 {k0, k1, k2,
 * global row, val}: a rank's distinct t keys (largest row, val = ~0) and f
 * keys (smallest row, val = count), each sent to the rank owning its key.
 *   route:  dedupe the rank's rows, write the records bucketed by owner into
 *           recs (owner order, t records first in each bucket; at most cap
 *           records), n_t / n_f (host, world entries) = the bucket sizes
 *   owner:  over every record this rank owns (all ranks' buckets for it,
 *           concatenated, each t-first): ret[k] = the f count summed over the
 *           ranks for t record k if its row is the key's largest, else 0;
 *           missing_row = the smallest f row whose key has no t row (~0 if
 *           none: the reference's "Number not included")
 *   counts: the sender, ret aligned with its own recs (nsent records):
 *           cnt[j] = 1 + ret of row j's record, start = exclusive scan of cnt
 *           (the rank's multiset positions, relative); total (host) = sum
 *   deal:   seg[c * seg_ld + start[j] + m] = t[c * t_ld + j], m < cnt[j]
 *   place:  buf holds multiset positions [pos0, pos0 + len) (column c at
 *           buf + c * buf_ld): even positions p to h1, odd to h2, at local
 *           row p / 2 - row0. */
int zkgpu_h1h2_shard_route(uint64_t *recs, uint64_t cap, uint32_t *n_t, uint32_t *n_f, const uint64_t *f,
                           uint64_t f_ld, const uint64_t *t, uint64_t t_ld, uint64_t nrows, uint64_t row0, uint32_t dim,
                           uint32_t world);
int zkgpu_h1h2_shard_owner(uint64_t *ret, const uint64_t *recs, uint64_t nrec, uint32_t dim, uint64_t *missing_row);
int zkgpu_h1h2_shard_counts(uint32_t *start, uint32_t *cnt, uint64_t *total, const uint64_t *sent, const uint64_t *ret,
                            uint64_t nsent, uint64_t nrows, uint64_t row0);
int zkgpu_h1h2_shard_deal(uint64_t *seg, uint64_t seg_ld, const uint64_t *t, uint64_t t_ld, const uint32_t *start,
                          const uint32_t *cnt, uint64_t nrows, uint32_t dim);
int zkgpu_h1h2_shard_place(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *buf,
                           uint64_t buf_ld, uint64_t pos0, uint64_t len, uint64_t row0, uint32_t dim);

/* ---- device memory (the host orchestrator owns HBM through these) -------- */
int zkgpu_dev_malloc(void **ptr, uint64_t bytes);
/* free / total HBM of the bound device (hipMemGetInfo) */
int zkgpu_device_memory(uint64_t *free_bytes, uint64_t *total_bytes);
int zkgpu_dev_free(void *ptr);
int zkgpu_memcpy_h2d(void *dst, const void *src, uint64_t bytes);
int zkgpu_memcpy_d2h(void *dst, const void *src, uint64_t bytes);
int zkgpu_memcpy_d2d(void *dst, const void *src, uint64_t bytes);
int zkgpu_memset_dev(void *dst, int value, uint64_t bytes);

/* ---- STARK stage primitives (device-resident, column-major sections) ------
 * Section table for the expression programs: base pointer + leading
 * dimension per eSection (include/zkgpu_zxp.h SEC_*), the device analogue of
 * the reference's mapOffsets/mapSectionsN (stark_info.cpp:473-482). */
typedef struct {
    uint64_t *sec[12];
    uint64_t ld[12];    /* leading dimension = rows allocated per column */
    uint32_t ncols[12]; /* columns allocated (bounds-checked at launch) */
} zkgpu_sections;

/* Executor stand-in for synthetic traces: column cols[k] of a column-major
 * buffer gets the deterministic pseudo-random elements rand(seed, stream, col, row). */
int zkgpu_rand_cols_dev(uint64_t *base, uint64_t ld, const uint32_t *cols, uint32_t ncols, uint64_t nrows,
                        uint64_t seed, uint64_t stream);
/* the same for a row block of a 2^log_n-row domain: local row r of the
 * buffer gets global row (row0 + r) mod 2^log_n (halo rows after a block wrap
 * to the domain's first rows) */
int zkgpu_rand_cols_rows_dev(uint64_t *base, uint64_t ld, const uint32_t *cols, uint32_t ncols, uint64_t row0,
                             uint64_t nrows, uint32_t log_n, uint64_t seed, uint64_t stream);

/* Rows of selected columns between column-major device buffers -- the halo
 * refresh, shifted-store spill and block copies of the row-sharded prover
 * (host/sharded_starks.hpp): for k < ncols, j < nrows
 *   dst[dcol_k * dst_ld + dst_row0 + j] = src[scol_k * src_ld + (src_row0 + j) mod 2^src_log_mod]
 * with dcol_k = dst_cols[k] (k when dst_cols is NULL), likewise scol_k;
 * src_log_mod = 0: no wrap.  The column lists are host arrays. */
int zkgpu_copy_rows_dev(uint64_t *dst, uint64_t dst_ld, uint64_t dst_row0, const uint32_t *dst_cols,
                        const uint64_t *src, uint64_t src_ld, uint64_t src_row0, uint32_t src_log_mod,
                        const uint32_t *src_cols, uint32_t ncols, uint64_t nrows);

/* Steps::step*_parser_first (steps.hpp:21-58; used at starks.cpp:73,155,193,
 * 241,371): evaluate one expression program (include/zkgpu_zxp.h) over every
 * row of its domain (2^log_dom rows).  instr/opnd are host arrays (uploaded),
 * challenges (8 x 3), publics and evals are host arrays; xdiv/xdivw are
 * device arrays (2n x 3 interleaved) for the FRI program, else NULL;
 * extend_bits sizes zhInv (zhInv.cpp:7-31); x_start = 1 (n domain) or 7 (2n). */
int zkgpu_zxp_eval_dev(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd, uint32_t n_tmp1,
                       uint32_t n_tmp3, const zkgpu_sections *sections, uint32_t log_dom, const uint64_t *challenges,
                       const uint64_t *publics, uint32_t n_publics, const uint64_t *evals, uint32_t n_evals,
                       const uint64_t *xdiv, const uint64_t *xdivw, uint32_t extend_bits, uint64_t x_start);

/* The same over ONE ROW BLOCK of a row-sharded domain (the
 * quotient and FRI programs run on the rows a GPU owns after the column ->
 * row exchange).  Rows 0 .. 2^log_rows - 1 of every section are evaluated;
 * x_i = x_start * w_{2^log_domain}^i (x_start = 7 * w^row0 for a block
 * starting at global row row0), zhInv uses N = 2^(log_domain - extend_bits)
 * (row0 must be a multiple of 2^extend_bits), and a read at row shift s >= 0
 * does not wrap: the caller stores the next block's first s rows (the halo)
 * after the block, so every section's ld >= 2^log_rows + s.  A store at row
 * shift s likewise writes local row i + s: its last s rows land in the halo,
 * and the caller moves them to the next block (host/sharded_starks.hpp). */
int zkgpu_zxp_eval_block_dev(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd, uint32_t n_tmp1,
                             uint32_t n_tmp3, const zkgpu_sections *sections, uint32_t log_rows, uint32_t log_domain,
                             const uint64_t *challenges, const uint64_t *publics, uint32_t n_publics,
                             const uint64_t *evals, uint32_t n_evals, const uint64_t *xdiv, const uint64_t *xdivw,
                             uint32_t extend_bits, uint64_t x_start);

/* Host-only compiler behind zkgpu_zxp_eval_dev (include/zkgpu_zxp.h,
 * "compiled programs"): folds the row-constant operands (challenges 8 x 3,
 * publics, evals n_evals x 3, literals) into linear-combination instructions
 * with at most max_terms terms each (0 = default 64, cap 256) and packs the
 * temporaries.  The output arrays stay valid until the next call on the same
 * thread.  No GPU needed; used by the tests to check the compiled program
 * against the source program on the CPU oracle. */
int zkgpu_zxp_compile(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd, uint32_t n_tmp1,
                      uint32_t n_tmp3, const uint64_t *challenges, const uint64_t *publics, uint32_t n_publics,
                      const uint64_t *evals, uint32_t n_evals, uint32_t max_terms, zxp_compiled *out);

/* Diagnostics for the run-time compiled expression kernels (csrc/zxp_jit.hip):
 * compile a program exactly as zkgpu_zxp_eval_dev does and write the
 * generated straight-line HIP kernel source into buf (truncated to buflen);
 * with rtc_check != 0 also compile it for gfx950 with hiprtc (or find it in
 * the on-disk code-object cache; rtc_check = 2 also writes the code object to
 * $ZKGPU_ZXP_JIT_DUMP).  rtc_check = 3 only queries the cache: returns 1 when
 * the compiled kernel is on disk, 0 when not.  No GPU needed.
 * Returns the source length (>= 0) or an error code. */
int zkgpu_zxp_jit_source(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd, uint32_t n_tmp1,
                         uint32_t n_tmp3, const uint64_t *challenges, const uint64_t *publics, uint32_t n_publics,
                         const uint64_t *evals, uint32_t n_evals, char *buf, uint64_t buflen, int rtc_check);

/* Polinomial::calculateZ(z, num, den) (polinomial.hpp:586-607), F_p^3 columns
 * (3 consecutive columns of ld each).  *closes = 1 iff z[n-1]*num[n-1]/den[n-1] == 1
 * (the reference's zkassert). */
int zkgpu_calculate_z_dev(uint64_t *z, uint64_t z_ld, const uint64_t *num, uint64_t num_ld, const uint64_t *den,
                          uint64_t den_ld, uint64_t n, int *closes);
/* One row block of the same grand product (the row-sharded prover: each rank
 * its block, then a scan of the W block totals): z[i] = z0 * prod_{j<i}
 * num[j] / den[j] for i < n; total (host, canonical) = z0 * prod_{j<n}
 * num[j] / den[j].  calculateZ over the whole domain is z0 = 1, closes iff
 * total == 1. */
int zkgpu_calculate_z_block_dev(uint64_t *z, uint64_t z_ld, const uint64_t *num, uint64_t num_ld, const uint64_t *den,
                                uint64_t den_ld, uint64_t n, const uint64_t z0[3], uint64_t total[3]);
/* Every grand product of a stage (starks.cpp:165-189: calculateZ per
 * permutation / plookup / connection context) in one round trip: request k is
 * zkgpu_calculate_z_dev's (z, z_ld, num, num_ld, den, den_ld) over the same n;
 * closes[k] as there.  One read-back of the nz totals instead of nz. */
typedef struct zkgpu_z_req {
    uint64_t *z;
    uint64_t z_ld;
    const uint64_t *num;
    uint64_t num_ld;
    const uint64_t *den;
    uint64_t den_ld;
} zkgpu_z_req;
int zkgpu_calculate_z_many_dev(const zkgpu_z_req *req, uint32_t nz, uint64_t n, int *closes);

/* Starks::evmap (starks.cpp:556-669): evals[e] = sum_{k<n} L(k) * pol_e[k << extend_bits],
 * L = lev or lpev (device, 3 columns of ld l_ld).  cols = host array of device
 * column pointers (first column of each polynomial), lds / dims / primes per
 * entry.  evals_out: host (n_ev x 3). */
int zkgpu_evmap_dev(uint64_t *evals_out, const uint64_t *const *cols, const uint64_t *lds, const uint32_t *dims,
                    const uint32_t *primes, uint32_t n_ev, const uint64_t *lev, const uint64_t *lpev, uint64_t l_ld,
                    uint64_t n, uint32_t extend_bits);

/* xDivXSubXi / xDivXSubWXi (starks.cpp:344-366) over x_k = 7 w_{2n}^k, k < 2^n_bits_ext;
 * w = Goldilocks::w(n_bits).  Outputs interleaved (2n x 3), device. */
int zkgpu_xdivxsub_dev(uint64_t *xdiv, uint64_t *xdivw, const uint64_t xi[3], uint32_t n_bits, uint32_t n_bits_ext);
/* The same for rows [row0, row0 + nrows) of the extended domain only, written
 * at their places (xdiv + 3 row0 ...): a row-sharded prover's block. */
int zkgpu_xdivxsub_rows_dev(uint64_t *xdiv, uint64_t *xdivw, const uint64_t xi[3], uint32_t n_bits,
                            uint32_t n_bits_ext, uint64_t row0, uint64_t nrows);
/* LEv / LpEv (starks.cpp:308-324: INTT_N of the powers of xi and of w_N xi),
 * rows [row0, row0 + nrows) in closed form: LEv[k] = ((1 - xi^N) / N) x_k /
 * (x_k - xi) with x_k = w_N^k (LpEv: w_N xi) -- the same field values, row by
 * row, so each rank computes only its own rows.  lev / lpev: 3 columns of
 * leading dimension ld holding rows row0.. at offset 0.  Fails
 * (ZKGPU_ERR_ARG) when xi lies in the base field, where a denominator may
 * vanish: interpolate (zkgpu_ext_powers_dev + zkgpu_gl_ntt_dev) instead. */
int zkgpu_lagrange_xi_rows_dev(uint64_t *lev, uint64_t *lpev, uint64_t ld, const uint64_t xi[3], uint32_t n_bits,
                               uint64_t row0, uint64_t nrows);

/* base^k for k < n into 3 columns of ld (LEv / LpEv, starks.cpp:308-324) */
int zkgpu_ext_powers_dev(uint64_t *out, uint64_t ld, const uint64_t base[3], uint64_t n);

/* cols[c][k] *= base^k for k < n, c < ncols (canonical outputs): the coset
 * shift of coefficient vectors (the shift^i multiply of
 * NTT_Goldilocks::extendPol, starks.cpp:53), used to move the quotient
 * pieces between coset-scaled and plain coefficients. */
int zkgpu_scale_by_powers_dev(uint64_t *cols, uint64_t ld, uint32_t ncols, uint64_t n, uint64_t base);

/* quotient split (starks.cpp:266-281): qq2 col 3p+d row k = qq1 col d row pN+k * shift_in^p, k < n */
int zkgpu_qsplit_dev(uint64_t *qq2, uint64_t ld2, const uint64_t *qq1, uint64_t ld1, uint64_t n, uint32_t q_deg,
                     uint64_t shift_in);
/* the same for dim input columns into output columns stride*p + d (d < dim
 * <= stride): a column owner of the row-sharded prover splits its one
 * quotient column (dim 1, stride 3) */
int zkgpu_qsplit_cols_dev(uint64_t *qq2, uint64_t ld2, const uint64_t *qq1, uint64_t ld1, uint64_t n, uint32_t q_deg,
                          uint64_t shift_in, uint32_t dim, uint32_t stride);

/* plookup h1/h2 (Polinomial::calculateH1H2_opt1 / _opt3, polinomial.hpp:349-583,
 * called at starks.cpp:104-127): f, t, h1, h2 are n-row columns of dimension
 * dim (1, or 3 = three column-major components ld apart).  Every table row
 * starts with multiplicity 1; each f value adds one to the LAST table row with
 * the same (canonical) value; the multiset in table order is dealt
 * alternately into h1 and h2.  An f value absent from t returns ZKGPU_ERR_ARG
 * ("Number not included", the reference exits) with *missing_row = the first
 * such f row; otherwise *missing_row = UINT64_MAX. */
int zkgpu_h1h2_dev(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *f, uint64_t f_ld,
                   const uint64_t *t, uint64_t t_ld, uint64_t n, uint32_t dim, uint64_t *missing_row);

/* 3 ext columns (ld) -> interleaved n x 3 (the FRI polynomial layout, friProve.cpp) */
int zkgpu_cols3_to_interleaved_dev(uint64_t *out, const uint64_t *cols, uint64_t ld, uint64_t n);

/* MerkleTreeGL::getGroupProof for a row-major device source (FRI trees) */
int zkgpu_gl_merkle_open_rows_dev(uint64_t *vals_out, uint64_t *sibs_out, const uint64_t *nodes, const uint64_t *src,
                                  uint64_t ncols, uint64_t nrows, const uint64_t *idx, uint64_t nq);

/* The query phase's openings of several trees in one round trip
 * (friProve.cpp:195-232 -- every tree's getGroupProof at its query indices):
 * request k is zkgpu_gl_merkle_open_dev (rows = 0: src column-major, ld) or
 * zkgpu_gl_merkle_open_rows_dev (rows = 1: src row-major, ld ignored) with the
 * same arguments and output layout; one index upload, the n kernels, one
 * download, one synchronisation.  Every index is checked before anything is
 * queued. */
typedef struct zkgpu_open_req {
    uint64_t *vals_out, *sibs_out;
    const uint64_t *nodes, *src;
    uint64_t ld, ncols, nrows;
    const uint64_t *idx;
    uint64_t nq;
    uint32_t rows;
} zkgpu_open_req;
int zkgpu_gl_merkle_open_many(const zkgpu_open_req *req, uint32_t n);

/* ---- arithmetic self-test hook -----------------------------------------------
 * Runs one device field operation elementwise on arbitrary u64 inputs
 * (including non-canonical values >= p) and stores canonical results:
 * op 0 a+b, 1 a-b, 2 a*b, 3 -a, 4 a*2^12, 5 a*2^48, 6 a*2^84, 7 a*2^100,
 * 8 a^7, 9 cubic-extension a*b (a, b, out are n x 3).  Used by the parity
 * tests to pin the arithmetic core against big-integer references. */
int zkgpu_gl_field_selftest_dev(uint64_t *out, const uint64_t *a, const uint64_t *b, uint64_t n, int op);

/* The same for the helpers whose final correction runs behind a wave-uniform
 * branch (csrc/gl_rb.hpp; the NTT pass butterflies and the Poseidon S-box,
 * MDS and dot-product reductions use them), and every shift-multiply:
 * op 0 gl_add_rb(a, b), 1 gl_sub_rb(a, b), 2 gl_mul_rb(a, b),
 * 3 gl_reduce128_rb(lo = a, hi = b), 4 gl_reduce96_small_rb(lo = a, hl = b mod 2^32),
 * 5 dot3_fin_rb(A0 = a, A1 = b, A2 = c), 6 mul2e_rb<e>(a), 7 mul2e<e>(a) (0 <= e < 192),
 * 8 the Poseidon S-box a^7 (pow7), 9 its squaring gl_sqr3(a),
 * 10 gl_reduce128(lo = a, hi = b), 11 Dot3::fin(A0 = a, A1 = b, A2 = c).
 * Canonical results; c is read by ops 5 and 11 only. */
int zkgpu_gl_field_selftest_rb_dev(uint64_t *out, const uint64_t *a, const uint64_t *b, const uint64_t *c, uint64_t n,
                                   int op, int e);

/* ---- live kernel profiling --------------------------------------------------
 * With profiling on, every kernel launch is bracketed by HIP events recorded
 * on the launch stream, tagged with the kernel name and its algorithmic bytes
 * (each input element read once, each output element written once).
 * zkgpu_prof_query synchronises the stream and returns, for one kernel name,
 * the launch count, summed device time (ms) and summed algorithmic bytes.
 * Replaces nothing in the reference (its TimerStart/TimerStopAndLog host
 * timers, starks.cpp:49-403, are kept by the host adapter). */
int zkgpu_prof_enable(int on);
int zkgpu_prof_reset(void);
int zkgpu_prof_query(const char *kernel, uint64_t *launches, double *total_ms, double *total_bytes);
/* names of kernels seen since the last reset, '\n'-separated, into buf */
int zkgpu_prof_kernels(char *buf, uint64_t buflen);

/* Stream marks (no reference counterpart: the reference times its stages on
 * the CPU, TimerStart / TimerStopAndLog around synchronous code): the host
 * prover's stage timers without a device synchronisation per stage.
 * zkgpu_mark records event `slot` (< ZKGPU_MARKS) on the library stream;
 * zkgpu_mark_elapsed waits for event b and returns the milliseconds from
 * event a to event b. */
#define ZKGPU_MARKS 256
int zkgpu_mark(uint32_t slot);
int zkgpu_mark_elapsed(uint32_t a, uint32_t b, double *ms);

#ifdef __cplusplus
}
#endif
#endif /* ZKGPU_H */
