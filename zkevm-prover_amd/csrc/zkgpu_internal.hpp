// Internal state of libzkgpu (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zkgpu.h"
#include "../../include/zkgpu_zxp.h"

namespace zk {

constexpr uint32_t NTT_MAX_PASSES = 4;  // log2 n <= 32 at radix <= 2^8
constexpr uint32_t TW_MAX_LOG = 28;     // big-twiddle base omega_{2^28}
constexpr uint32_t TW_LEVEL_BITS = 14;
constexpr uint64_t TW_LEVEL_SIZE = 1ULL << TW_LEVEL_BITS;
constexpr uint32_t POST_BITS = 12;  // LDE shift-power tables: lo 4096 entries

struct Workspace {
    void *ptr = nullptr;
    size_t bytes = 0;
};

struct Ctx {
    int device = -1;
    bool ready = false;
    hipStream_t stream = nullptr;  // launches go here (zkgpu_set_stream)
    // direction 0 = forward, 1 = inverse
    uint64_t *rt_small[2] = {nullptr, nullptr};  // omega_4096^k, k < 4096 (this direction)
    uint64_t *tw_lo[2] = {nullptr, nullptr};     // omega_{2^28}^i, i < 2^14
    uint64_t *tw_hi[2] = {nullptr, nullptr};     // omega_{2^28}^(2^14 i)
    // LDE post-scale tables (1/n * 7^k), cached per log n
    uint32_t post_logn = 0;
    uint64_t *post_lo = nullptr;
    uint64_t *post_hi = nullptr;
    // scratch workspaces
    Workspace ws[7];  // 0-3 NTT / staging, 4 H1H2 scratch, 5 rocPRIM temp, 6 ZXP segment carries
    // Poseidon constants on device
    uint64_t *poseidon_rc = nullptr;
};

Ctx &ctx();
int set_error(int code, const char *fmt, ...);
int check_launch(const char *what);
int check_hip(hipError_t e, const char *what);
// grow-only scratch buffer i
uint64_t *workspace(int i, size_t bytes);

// host-side scalar Goldilocks (setup values only; all bulk math is on the GPU)
uint64_t h_mul(uint64_t a, uint64_t b);
uint64_t h_pow(uint64_t a, uint64_t e);
uint64_t h_inv(uint64_t a);
uint64_t h_w(uint32_t n);

// ---- live kernel profiling (HIP events on the launch stream; zkgpu_prof_*)
// prof_begin/prof_end bracket one kernel launch; bytes = algorithmic bytes
// (each input element read once + each output element written once).
bool prof_on();
void prof_begin(hipStream_t s);
void prof_end(const char *kernel, double bytes, hipStream_t s);

// ---- ntt.hip
int ntt_columns(Ctx &c, uint64_t *dst, uint64_t dst_ld, const uint64_t *src, uint64_t src_ld, uint64_t src_valid,
                uint64_t *tmp, uint64_t tmp_ld, uint32_t logn, uint64_t ncols, int inverse, const uint64_t *post_lo,
                const uint64_t *post_hi, uint32_t post_bits, uint64_t post_base, uint64_t post_scale, hipStream_t s);
void rows_to_cols(const uint64_t *in, uint64_t *out, uint64_t nrows, uint64_t ncols, uint64_t ld, hipStream_t s);
void cols_to_rows(const uint64_t *in, uint64_t *out, uint64_t nrows, uint64_t ncols, uint64_t ld, hipStream_t s);
void fill_powers(uint64_t *out, uint64_t base, uint64_t step, uint64_t scale, uint64_t count, hipStream_t s);
// 3-pass LDE 2^logn -> 2^(logn+1) (ntt.hip "3-pass LDE"); t1: 2^logn words per column
bool lde3_supported(uint32_t logn, uint32_t loge);
int lde3_columns(Ctx &c, uint64_t *out, uint64_t ld_out, const uint64_t *in, uint64_t ld_in, uint64_t *t1,
                 uint32_t logn, uint64_t ncols, hipStream_t s);

// ---- poseidon.hip
int poseidon_batch(uint64_t *out, const uint64_t *in, uint64_t n, int full, hipStream_t s);
int merkle_leaves_cols(uint64_t *digests, const uint64_t *src, uint64_t ncols, uint64_t nrows, uint64_t ld,
                       hipStream_t s, const uint64_t *src2 = nullptr, uint64_t split = 0);
int merkle_leaves_rows(uint64_t *digests, const uint64_t *src, uint64_t ncols, uint64_t nrows, hipStream_t s);
int merkle_levels(uint64_t *nodes, uint64_t nrows, hipStream_t s);
int merkle_open_cols(uint64_t *vals, uint64_t *sibs, const uint64_t *nodes, const uint64_t *src, uint64_t ncols,
                     uint64_t nrows, uint64_t ld, const uint64_t *idx, uint64_t nq, hipStream_t s);

// ---- h1h2.hip, row-sharded calculateH1H2 (host/sharded_starks.hpp)
int h1h2_shard_route(uint64_t *recs, uint64_t cap, uint32_t *n_t, uint32_t *n_f, const uint64_t *f, uint64_t f_ld,
                     const uint64_t *t, uint64_t t_ld, uint64_t n, uint64_t row0, uint32_t dim, uint32_t world,
                     hipStream_t s);
int h1h2_shard_owner(uint64_t *ret, const uint64_t *recs, uint64_t nrec, uint32_t dim, uint64_t *miss_row,
                     hipStream_t s);
int h1h2_shard_counts(uint32_t *start, uint32_t *cnt, uint64_t *total, const uint64_t *sent, const uint64_t *ret,
                      uint64_t nsent, uint64_t n, uint64_t row0, hipStream_t s);
int h1h2_shard_deal(uint64_t *seg, uint64_t seg_ld, const uint64_t *t, uint64_t t_ld, const uint32_t *start,
                    const uint32_t *cnt, uint64_t n, uint32_t dim, hipStream_t s);
int h1h2_shard_place(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *buf, uint64_t buf_ld,
                     uint64_t pos0, uint64_t len, uint64_t row0, uint32_t dim, hipStream_t s);

// ---- fri.hip
int fri_fold(uint64_t *out, const uint64_t *pol, uint32_t pol_bits, uint32_t out_bits, const uint64_t sx[3],
             uint64_t shift_inv, hipStream_t s);
int fri_fold_rows(uint64_t *out, const uint64_t *rows, uint64_t g0, uint64_t n_local, uint32_t pol_bits,
                  uint32_t out_bits, const uint64_t sx[3], uint64_t shift_inv, hipStream_t s);
int fri_transpose(uint64_t *aux, const uint64_t *pol, uint64_t degree, uint32_t tbits, hipStream_t s);

// ---- stark.hip
// Pre-decoded ZXP instruction (built on the host by zkgpu_zxp_eval_dev): every
// operand is resolved to a source kind plus a ready pointer / shift / stride /
// immediate, so the kernel fetches one 128-byte record per instruction with
// wave-uniform scalar loads and no dependent descriptor or section lookups.
enum { DK_T1 = 0, DK_T3, DK_C1, DK_C3, DK_IMM1, DK_IMM3, DK_X, DK_I3, DK_ZI };
struct alignas(16) ZOp {
    uint32_t op, ka, kb, kd;
    const uint64_t *pa, *pb;
    uint64_t *pd;
    int32_t ia, ib, id;  // T*: slot offset (slot * 64); C*: row shift; ZI: index mask
                         // DOT: ia = first term, ib = term count; ima/imb = constant limbs (9 u32)
    uint32_t lda, ldb, ldd;
    uint64_t ima[3], imb[3];
    uint64_t pad[2];
};
static_assert(sizeof(ZOp) == 128, "ZOp is two 64-byte scalar loads");

// ZXP_DOT term: source (a column at a row shift, or an LDS temp slot
// component) and its F_p^3 coefficient as Dot3 limbs (3 components x 6).
struct alignas(16) ZTerm {
    uint32_t kind;  // DK_C1 or DK_T1
    int32_t ii;     // C1: row shift; T1: LDS offset (slot * 64)
    const uint64_t *ptr;
    uint32_t c[3][6];
    uint32_t pad[2];
};
static_assert(sizeof(ZTerm) == 96, "ZTerm is 96 bytes");

struct ZxpLaunch {
    uint64_t *sec[SEC_COUNT];
    uint64_t ld[SEC_COUNT];
    const ZOp *prog;  // device, n_instr records
    const ZTerm *terms;  // device, DOT terms
    uint32_t n_instr, n_tmp1, n_tmp3;
    uint32_t logdom;    // rows evaluated
    uint32_t logomega;  // x_i = x_start * omega_{2^logomega}^i
    uint32_t wrap;      // shifted reads wrap mod 2^logdom (else halo rows follow)
    const uint64_t *challenges, *publics, *evals;  // device
    const uint64_t *xdiv, *xdivw;                  // device (2n domain) or null
    const uint64_t *zhinv;                         // device, 2^eb entries
    uint32_t zhinv_mask;
    uint64_t x_start;
    double bytes;  // algorithmic bytes for profiling
};
// ---- zxp_jit.hip: run-time compiled straight-line expression kernels
struct ZxpJitIn {
    const zxp_instr *ins;  // compiled program (zkgpu_zxp_compile)
    uint32_t n_instr;
    const zxp_operand *opnd;
    uint32_t n_opnd;
    const zxp_term *terms;
    const uint64_t *csts;
    uint32_t n_tmp1, n_tmp3;
    const zkgpu_sections *sections;
    uint32_t log_dom;   // rows evaluated
    uint32_t log_omega; // x_i = x_start * omega_{2^log_omega}^i
    uint32_t wrap;      // shifted reads wrap mod 2^log_dom (else halo rows follow)
    const uint64_t *challenges, *publics, *evals;  // host
    const uint64_t *xdiv, *xdivw, *zh_dev;         // device
    uint32_t zmask;
    uint64_t x_start;
    double bytes;
    uint32_t dot_loop_min;  // DOTs with at least this many column terms loop over a table
    uint32_t waves_per_eu;  // occupancy hint for the compiler (0: none)
    uint32_t force_split;   // code blocks / limb chunks even below the size threshold (segments)
    const uint64_t *scratch;  // columns of section ZXP_SEC_SCRATCH (segments, csrc/zxp_segment.hpp)
    uint64_t scratch_ld;
};
// 0 launched, 1 shape unsupported (run the interpreter), < 0 error
int zxp_jit_run(const ZxpJitIn &in, hipStream_t s);
// Dot3 limbs of a canonical coefficient c: 22/21/21-bit limbs of c and of
// c * 2^32 mod p (csrc/gl_device.hpp Dot3::term)
inline void zxp_limbs6(uint64_t c, uint32_t out[6])
{
    const uint64_t v[2] = {c, h_mul(c, 1ULL << 32)};
    for (int h = 0; h < 2; h++) {
        out[3 * h] = (uint32_t)(v[h] & ((1u << 22) - 1));
        out[3 * h + 1] = (uint32_t)((v[h] >> 22) & ((1u << 21) - 1));
        out[3 * h + 2] = (uint32_t)(v[h] >> 43);
    }
}

int rand_cols(uint64_t *base, uint64_t ld, const uint32_t *cols_dev, uint32_t ncols, uint64_t nrows, uint64_t seed,
              uint64_t stream, uint64_t row0, uint64_t rmask, hipStream_t s);
int copy_rows(uint64_t *dst, uint64_t dld, uint64_t drow0, const uint32_t *dcols, const uint64_t *src, uint64_t sld,
              uint64_t srow0, uint64_t smask, const uint32_t *scols, uint32_t ncols, uint64_t nrows, hipStream_t s);
int zxp_eval(const ZxpLaunch &L, hipStream_t s);
size_t calculate_z_scratch_words(uint64_t n);
int calculate_z(uint64_t *z, uint64_t z_ld, const uint64_t *num, uint64_t num_ld, const uint64_t *den,
                uint64_t den_ld, uint64_t n, const uint64_t z0[3], uint64_t *scratch, uint64_t *total_dev, hipStream_t s);
size_t evmap_group_size();
uint32_t evmap_group_width();
uint64_t evmap_rows_per_block();
int evmap_groups(uint64_t *evals, const void *groups_dev, uint32_t n_groups, uint32_t width, uint32_t unroll,
                 const int32_t *subs_dev,
                 uint32_t n_ev, uint32_t n_sub, const uint64_t *lev, const uint64_t *lpev, uint64_t l_ld, uint64_t n, uint32_t eb,
                 uint64_t *partial, hipStream_t s);
int xdivxsub(uint64_t *xdiv, uint64_t *xdivw, const uint64_t xi[3], uint64_t w, uint32_t logn, hipStream_t s);
int xdivxsub_rows(uint64_t *xdiv, uint64_t *xdivw, const uint64_t xi[3], uint64_t w, uint32_t logn, uint64_t row0,
                  uint64_t nrows, hipStream_t s);
int xdiv_rows(uint64_t *out0, uint64_t *out1, uint64_t ld, int interleaved, const uint64_t a0[3],
              const uint64_t a1[3], uint64_t shift, const uint64_t scale[3], uint32_t logn, uint64_t row0,
              uint64_t nrows, hipStream_t s);
int ext_powers(uint64_t *out, uint64_t ld, const uint64_t base[3], uint64_t n, hipStream_t s);
int scale_powers(uint64_t *cols, uint64_t ld, uint32_t ncols, uint64_t n, uint64_t base, hipStream_t s);
int qsplit(uint64_t *qq2, uint64_t ld2, const uint64_t *qq1, uint64_t ld1, uint64_t n, uint32_t qdeg,
           uint64_t shift_in, uint32_t dim, uint32_t stride, hipStream_t s);
int cols3_to_interleaved(uint64_t *out, const uint64_t *cols, uint64_t ld, uint64_t n, hipStream_t s);
int h1h2(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *f, uint64_t f_ld,
         const uint64_t *t, uint64_t t_ld, uint64_t n, uint32_t dim, uint64_t *missing_row, hipStream_t s);
int merkle_open_strided(uint64_t *vals, uint64_t *sibs, const uint64_t *nodes, const uint64_t *src, uint64_t ncols,
                        uint64_t nrows, uint64_t row_stride, uint64_t col_stride, const uint64_t *idx, uint64_t nq,
                        hipStream_t s);

}  // namespace zk
