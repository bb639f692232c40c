/*
 * zkgpu_stark.h -- C-ABI of libzkgpu_stark, the host-side STARK prover
 * (a C++ restatement of Starks::genProof, starks.cpp:9-404, and
 * FRIProve::prove, friProve.cpp:5-190) that drives the MI355X kernels only
 * through include/zkgpu.h.  The instance description plays the role of the
 * reference's StarkInfo (stark_info.hpp:269-336) + Steps (steps.hpp).
 *
 * Proof output: one flat u64 buffer in the reference's zkin order
 * (proof2zkinStark.cpp:8-82), canonical values:
 *   root1[4] root2[4] root3[4] root4[4] evals[n_ev*3]
 *   for si = 1 .. n_fri_steps-1:
 *       s{si}_root[4]  s{si}_vals[Q][3*2^(steps[si-1]-steps[si])]  s{si}_siblings[Q][steps[si]][4]
 *   s0_vals1[Q][n_cm1] s0_vals2[Q][n_cm2] s0_vals3[Q][n_cm3] s0_vals4[Q][n_cm4] s0_valsC[Q][n_const]
 *   s0_siblings{1,2,3,4,C}[Q][n_bits_ext][4]
 *   finalPol[2^steps[last]][3]
 */
#ifndef ZKGPU_STARK_H
#define ZKGPU_STARK_H
#include <stdint.h>

#include "zkgpu_zxp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    const zxp_instr *instr;
    uint32_t n_instr;
    const zxp_operand *opnd;
    uint32_t n_opnd;
    uint32_t n_tmp1, n_tmp3;
} zkgpu_zxp_prog;

typedef struct {
    uint32_t n_bits, n_bits_ext, n_queries, n_fri_steps;
    uint32_t fri_steps[32];
    uint32_t n_cm1, n_cm2, n_cm3, n_cm4, n_tmp, n_const, n_publics, q_deg, l_first, n_k;
    uint64_t seed;
    uint32_t n_random_cols;
    const uint32_t *random_cols; /* cm1 columns filled by the trace generator */
    uint32_t n_zctx;
    const uint32_t *zctx; /* (num tmp col, den tmp col, z cm3 col) triples */
    uint32_t n_ev;
    const uint32_t *ev; /* evMap (section_2ns, col, dim, prime) quads */
    zkgpu_zxp_prog step1, step2, step3prev, step42ns, step52ns;
    /* constant polynomials (setup; the reference loads them from the
     * zkevmConstPols file, starks.hpp:94-116): these columns are filled
     * pseudo-randomly (n_random_const = 0: columns 0 .. n_k-1), l_first gets
     * L_first, then step0 derives the rest on the N domain (may be empty) */
    uint32_t n_random_const;
    const uint32_t *random_const;
    zkgpu_zxp_prog step0;
    /* plookups (starkInfo.puCtx, starks.cpp:104-127): (f tmp col, t tmp col,
     * h1 cm2 col, h2 cm2 col, dim) quintuples; h1/h2 are computed after step2 */
    uint32_t n_pu;
    const uint32_t *pu;
    /* post-Z stage-3 expressions (starks.cpp:193-208, Steps::step3_parser_first):
     * run after calculateZ, before the stage-3 LDE + commit (may be empty) */
    zkgpu_zxp_prog step3;
} zkgpu_stark_info;

/* allocate the HBM memory map, build the constant polynomials, their LDE and
 * the constant tree (the reference loads these from files; setup, untimed).
 * Memory plan ZKGPU_MEM_AUTO (below). */
int zkgpu_stark_create(void **handle, const zkgpu_stark_info *info);

/* HBM plans of the single-GPU prover (the reference allocates one memory map
 * for the prover's life and reuses sections as scratch, prover.cpp:94,
 * starks.cpp:53,105):
 *   RESIDENT  every section of both domains held for the prover's life: the
 *             trace survives a proof (prove may run again on it).
 *   LEAN      one arena whose regions follow the sections' lifetimes within a
 *             proof: cm1's stage-1 extension is hashed and dropped, the
 *             n-domain sections die after stage 3, cm3 and (before stage 4)
 *             cm1 are extended in place over their n-domain values, evmap
 *             reads the extended rows k << blowup (starks.cpp:308-333).  The
 *             proof consumes cm1_n: set_cm1 / witness before every prove
 *             (prove fails loudly otherwise); set_cm1_async is not offered.
 *             At the fork-9 widths and 2^23 rows: about 260 GB instead of 386.
 *   AUTO      RESIDENT when its plan fits the device's free HBM, else LEAN.
 * Proofs are bit-identical under every plan. */
enum { ZKGPU_MEM_AUTO = 0, ZKGPU_MEM_RESIDENT = 1, ZKGPU_MEM_LEAN = 2 };
int zkgpu_stark_create_ex(void **handle, const zkgpu_stark_info *info, uint32_t memory_plan);
/* the plan a single-GPU prover runs under (ZKGPU_MEM_RESIDENT / _LEAN) */
int zkgpu_stark_memory_mode(void *handle);
/* synthetic committed trace cm1_n (executor stand-in: PRNG columns + step1) */
int zkgpu_stark_witness(void *handle);
/* load cm1_n from a host row-major buffer (n rows x n_cm1), the reference's
 * commit-pols layout (commit_pols.hpp:18) */
int zkgpu_stark_set_cm1(void *handle, const uint64_t *rows);
/* queue the trace of the proof AFTER the next one: returns at once, the
 * trace crosses PCIe into a second cm1_n buffer (zkgpu_load_rows_async)
 * while the next zkgpu_stark_prove runs on the current cm1_n, and becomes
 * cm1_n when that prove returns.  `rows` must stay valid until then; a later
 * set_cm1 / set_cm1_async supersedes it.  Costs one more cm1_n (n x n_cm1
 * u64; a shard's rows on a sharded prover) of HBM.  On a sharded prover each
 * rank passes the whole row-major buffer and loads its own rows, as with
 * set_cm1. */
int zkgpu_stark_set_cm1_async(void *handle, const uint64_t *rows);
/* cm1_n back into a host row-major buffer (n rows x n_cm1; the inverse of
 * set_cm1).  Single-GPU prover only. */
int zkgpu_stark_get_cm1(void *handle, uint64_t *rows);
/* load the constant polynomials from a host row-major buffer (n rows x
 * n_const), the reference's .const file (ConstantPolsStarks, starks.hpp:94-116);
 * recomputes their LDE, tree and verkey */
int zkgpu_stark_set_const(void *handle, const uint64_t *rows);
/* set the public inputs (n_publics values; prover.cpp:480-560 computes them
 * from the executor's Main columns) */
int zkgpu_stark_set_publics(void *handle, const uint64_t *publics);
uint64_t zkgpu_stark_proof_len(void *handle);
int zkgpu_stark_prove(void *handle, uint64_t *proof_out);
int zkgpu_stark_verkey(void *handle, uint64_t out[4]);
int zkgpu_stark_publics(void *handle, uint64_t *out);
/* STARK_STEP_* timers of the last prove (starks.cpp:49-403 names):
 * names '\n'-separated into names_buf, milliseconds into ms; returns count */
int zkgpu_stark_timers(void *handle, char *names_buf, uint64_t names_len, double *ms, uint32_t max);
void zkgpu_stark_destroy(void *handle);
const char *zkgpu_stark_last_error(void);

/* ---- the Fiat-Shamir transcript the prover runs on the host, as the
 * reference's class Transcript (transcript.hpp:14-37, transcript.cpp:4-88):
 * Poseidon-GL sponge, 8-element rate, 4-element capacity.  Host code only
 * (no GPU, no zkgpu_init needed).  Inputs are any u64 (reduced mod p, as
 * Goldilocks::Element); outputs are canonical. */
typedef struct zkgpu_transcript zkgpu_transcript;
zkgpu_transcript *zkgpu_transcript_create(void);                              /* Transcript() */
int zkgpu_transcript_put(zkgpu_transcript *t, const uint64_t *in, uint64_t n); /* put, :4-29 */
int zkgpu_transcript_get_fields1(zkgpu_transcript *t, uint64_t *out);         /* getFields1, :39-55 */
int zkgpu_transcript_get_field(zkgpu_transcript *t, uint64_t out[3]);         /* getField, :31-37 */
/* getPermutations, :57-88: n indices of nbits bits each (nbits <= 63) */
int zkgpu_transcript_get_permutations(zkgpu_transcript *t, uint64_t *res, uint64_t n, uint64_t nbits);
void zkgpu_transcript_destroy(zkgpu_transcript *t);

/* ---- one proof sharded over the GPUs of a node (BASELINE
 * configs[4]: "the same BatchProof trace column-sharded across 8 x MI355X").
 * The reference proves on one host (Starks::genProof, starks.cpp:9-404); this
 * is the multi-GPU form of the same proof, bit-identical to it.
 *
 * Point-to-point exchange between the ranks of a sharded prover: one grouped
 * batch of sends and receives of DEVICE buffers.  Operations with the same
 * peer and direction match in order on both sides; never peer == rank.  The
 * call returns once work enqueued afterwards on the zkgpu stream
 * (zkgpu_get_stream) sees the received bytes; the send buffers are not
 * modified before that either. */
typedef struct {
    int32_t peer;
    int32_t send; /* 1: send buf to peer; 0: receive into buf from peer */
    void *buf;    /* device pointer */
    uint64_t bytes;
} zkgpu_comm_op;

typedef struct {
    uint32_t rank, world; /* world a power of two */
    void *ctx;
    int (*exchange)(void *ctx, const zkgpu_comm_op *ops, uint32_t n_ops);
    /* optional (may be NULL): this rank has failed -- release the peers.  The
     * prover calls it when a sharded proof fails on this rank (a local error,
     * or an exchange it refuses), so that no peer waits for it: every later
     * exchange of the communicator then fails, on this rank at once and on the
     * peers at their next exchange (host shared memory) or within the
     * exchange deadline (RCCL). */
    int (*abort)(void *ctx);
} zkgpu_comm;

/* The RCCL implementation (ncclSend / ncclRecv inside ncclGroupStart/End,
 * enqueued on the zkgpu stream; xGMI between the GPUs of a node).  One rank
 * makes the id and hands it to the others (any side channel); every rank then
 * creates its communicator with its own rank.  librccl is opened at run time.
 * Each exchange waits for its transfers with a deadline (ZKGPU_COMM_TIMEOUT_S
 * seconds, default 120) while polling ncclCommGetAsyncError; on an error or
 * the deadline it calls ncclCommAbort (the transfer kernels exit) and fails,
 * and so does every later exchange: a rank whose peer failed or stopped
 * returns an error within the deadline instead of waiting forever. */
int zkgpu_comm_rccl_unique_id(uint8_t id[128]);
int zkgpu_comm_rccl_create(zkgpu_comm *comm, const uint8_t id[128], uint32_t world, uint32_t rank);
void zkgpu_comm_rccl_destroy(zkgpu_comm *comm);

/* Host shared-memory implementation for ranks that cannot use RCCL (several
 * processes sharing one GPU): POSIX shared memory `name` ("/..."), one
 * outbox of `capacity` bytes per rank and exchange, process-shared barriers.
 * Every rank calls create with the same name, world and capacity. */
int zkgpu_comm_host_create(zkgpu_comm *comm, const char *name, uint32_t world, uint32_t rank, uint64_t capacity);
void zkgpu_comm_host_destroy(zkgpu_comm *comm);

/* A prover whose extended (2n) domain is row-sharded over comm->world ranks:
 * rank r holds rows [r 2n/W, (r+1) 2n/W) of every extended section (plus the
 * next block's first 2^blowup rows), rows [r n/W, (r+1) n/W) of every n-domain
 * section (plus the next block's first rows up to the programs' largest row
 * shift), its share of the commitments' LDE columns, and the subtrees of its
 * rows.  Every rank calls the same functions in the same order
 * (witness / set_cm1 / set_const / set_publics / prove are collective) and
 * every rank's zkgpu_stark_prove returns the same proof, equal to
 * zkgpu_stark_create's.  comm is copied; comm->ctx must outlive the handle. */
int zkgpu_stark_create_sharded(void **handle, const zkgpu_stark_info *info, const zkgpu_comm *comm);
/* HBM one GPU holds at its peak for this description (its sections, the
 * transient setup copy of the constants, the library's workspaces): world 0
 * = zkgpu_stark_create, world W >= 1 = zkgpu_stark_create_sharded over W
 * ranks.  Host only, no GPU needed; both create calls fail loudly, before
 * allocating, when it exceeds the device's free memory. */
int zkgpu_stark_memory_plan(const zkgpu_stark_info *info, uint32_t world, uint64_t *bytes_per_gpu);
/* the same for a single-GPU prover (world 0) under memory plan RESIDENT or
 * LEAN (ZKGPU_MEM_*; AUTO = RESIDENT here: the choice needs a device) */
int zkgpu_stark_memory_plan_ex(const zkgpu_stark_info *info, uint32_t memory_plan, uint64_t *bytes);

#ifdef __cplusplus
}
#endif
#endif /* ZKGPU_STARK_H */
