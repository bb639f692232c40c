// STARK stage kernels for gfx950: expression programs, grand products,
// evaluations at xi, FRI-polynomial helpers, quotient split.
//
//   k_zxp_eval      Steps::step2prev / step3prev / step42ns / step52ns
//                   (steps.hpp:21-58; op semantics of
//                   zkevm.chelpers.step42ns.parser.cpp:24-784, step52ns.parser.cpp:9-226)
//                   as a uniform-control-flow interpreter: one thread per row,
//                   instructions and operand descriptors are wave-uniform
//                   (scalar loads, scalar branches), temporaries live in LDS
//                   slot-major (conflict-free), sections are column-major.
//   calculateZ      Polinomial::calculateZ (polinomial.hpp:586-607): per-row
//                   ratio num/den (chunked Montgomery batch inversion), then a
//                   3-phase parallel exclusive prefix product in F_p^3.
//   k_evmap         Starks::evmap (starks.cpp:556-669): sum_k L(k) pol[k << eb]
//   k_xdiv_rows     xDivXSub (starks.cpp:344-366), LEv / LpEv closed form
//   k_ext_powers    LEv / LpEv power sequences (starks.cpp:308-324)
//   k_qsplit        quotient split (starks.cpp:264-281)
// F_p^3 arithmetic is associative/commutative and exact, so any reduction
// order gives the reference's values bit for bit.
#include "gl_device.hpp"
#include "zkgpu_internal.hpp"
#include "../../include/zkgpu_zxp.h"

namespace zk {

// ---------------------------------------------------------------- F_p^3 inverse
// a * b = 1 with M(a) b = e0, M(a) = [[a0, a2, a1], [a1, a0+a2, a1+a2], [a2, a1, a0+a2]]
// (x^3 = x + 1); b = first column of adj(M) / det(M).
template <int K>
__device__ __forceinline__ uint64_t sqr_n(uint64_t x)
{
#pragma unroll
    for (int i = 0; i < K; i++) x = gl_sqr(x);
    return x;
}

// a^(p-2), p - 2 = (2^31 - 1) * 2^33 + (2^32 - 1): 64 squarings + 9 multiplications
__device__ __forceinline__ uint64_t gl_inv_base(uint64_t x)
{
    uint64_t t2 = gl_mul(gl_sqr(x), x);          // 2^2 - 1
    uint64_t t3 = gl_mul(gl_sqr(t2), x);         // 2^3 - 1
    uint64_t t6 = gl_mul(sqr_n<3>(t3), t3);      // 2^6 - 1
    uint64_t t12 = gl_mul(sqr_n<6>(t6), t6);     // 2^12 - 1
    uint64_t t24 = gl_mul(sqr_n<12>(t12), t12);  // 2^24 - 1
    uint64_t t30 = gl_mul(sqr_n<6>(t24), t6);    // 2^30 - 1
    uint64_t t31 = gl_mul(gl_sqr(t30), x);       // 2^31 - 1
    uint64_t t32 = gl_mul(gl_sqr(t31), x);       // 2^32 - 1
    return gl_mul(sqr_n<33>(t31), t32);
}

__device__ __forceinline__ gl3 gl3_inv(const gl3 &a)
{
    uint64_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2];
    uint64_t s02 = gl_add(a0, a2), s12 = gl_add(a1, a2);
    uint64_t c0 = gl_sub(gl_mul(s02, s02), gl_mul(s12, a1));
    uint64_t c1 = gl_sub(gl_mul(s12, a2), gl_mul(a1, s02));
    uint64_t c2 = gl_sub(gl_mul(a1, a1), gl_mul(s02, a2));
    uint64_t det = gl_add(gl_add(gl_mul(a0, c0), gl_mul(a2, c1)), gl_mul(a1, c2));
    uint64_t di = gl_inv_base(det);
    return gl3{{gl_mul(c0, di), gl_mul(c1, di), gl_mul(c2, di)}};
}

__device__ __forceinline__ gl3 ld3(const uint64_t *p0, uint64_t ld)
{
    return gl3{{p0[0], p0[ld], p0[2 * ld]}};
}

__device__ __forceinline__ void st3(uint64_t *p0, uint64_t ld, const gl3 &v)
{
    p0[0] = gl_canon(v.v[0]);
    p0[ld] = gl_canon(v.v[1]);
    p0[2 * ld] = gl_canon(v.v[2]);
}

// ---------------------------------------------------------------- PRNG columns
__device__ __forceinline__ uint64_t rand_u64(uint64_t seed, uint64_t stream, uint64_t col, uint64_t row)
{
    uint64_t x = seed ^ (stream << 56) ^ (col * 0x9E3779B97F4A7C15ULL) ^ (row * 0xC2B2AE3D27D4EB4FULL);
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return z >> 1;
}

// local row r holds global row (row0 + r) & rmask (a row block of a sharded
// domain, its halo rows wrapping to the domain's first rows)
__global__ void k_rand_cols(uint64_t *base, uint64_t ld, const uint32_t *cols, uint32_t ncols, uint64_t nrows,
                            uint64_t seed, uint64_t stream, uint64_t row0, uint64_t rmask)
{
    uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t k = blockIdx.y;
    if (r >= nrows || k >= ncols) return;
    uint32_t c = cols[k];
    base[(uint64_t)c * ld + r] = rand_u64(seed, stream, c, (row0 + r) & rmask);
}

// rows of selected columns between two column-major buffers (the halo and
// block exchanges of the row-sharded prover): dst column dcols[k] (k if
// null), rows drow0 + j  <-  src column scols[k] (k if null), rows
// (srow0 + j) & smask.  One wave covers 64 consecutive rows of one column.
__global__ void k_copy_rows(uint64_t *dst, uint64_t dld, uint64_t drow0, const uint32_t *dcols, const uint64_t *src,
                            uint64_t sld, uint64_t srow0, uint64_t smask, const uint32_t *scols, uint32_t ncols,
                            uint64_t nrows)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t k = blockIdx.y;
    if (j >= nrows || k >= ncols) return;
    const uint64_t dc = dcols ? dcols[k] : k, sc = scols ? scols[k] : k;
    dst[dc * dld + drow0 + j] = src[sc * sld + ((srow0 + j) & smask)];
}

// ---------------------------------------------------------------- ZXP interpreter
struct ZxpEnv {
    const ZOp *prog;
    const ZTerm *terms;
    uint32_t n_instr;
    uint32_t logdom;        // rows evaluated: 2^logdom
    uint32_t logomega;      // x_i = x_start * omega_{2^logomega}^i
    uint64_t rmask;         // shifted reads: (i + shift) & rmask (all ones = no wrap, halo rows provided)
    uint64_t x_start;
    const uint64_t *tw_lo;  // forward big twiddles (omega_2^28)
    const uint64_t *tw_hi;
};

constexpr int ZXP_THREADS = 64;

struct Val {
    gl3 v;
    int dim;
};

// Temp slot s of lane l lives at lds[s * 64 + l] (each wave access = 64
// consecutive u64); the host pre-multiplies slot indices by 64.
__device__ __forceinline__ Val zxp_load(const ZxpEnv &e, uint32_t kind, const uint64_t *ptr, int32_t ii, uint32_t ld,
                                        const uint64_t *imm, const uint64_t *lds, int lane, uint64_t i)
{
    Val r;
    r.dim = 1;
    r.v.v[1] = r.v.v[2] = 0;
    switch (kind) {
    case DK_T1: r.v.v[0] = lds[ii + lane]; break;
    case DK_T3: {
        const uint64_t *p = lds + ii + lane;
        r.v = gl3{{p[0], p[ZXP_THREADS], p[2 * ZXP_THREADS]}};
        r.dim = 3;
        break;
    }
    case DK_C1: r.v.v[0] = gload(ptr + ((i + (uint64_t)(int64_t)ii) & e.rmask)); break;
    case DK_C3: {
        const uint64_t *p = ptr + ((i + (uint64_t)(int64_t)ii) & e.rmask);
        r.v = gl3{{gload(p), gload(p + ld), gload(p + 2 * (uint64_t)ld)}};
        r.dim = 3;
        break;
    }
    case DK_IMM1: r.v.v[0] = imm[0]; break;
    case DK_IMM3: r.v = gl3{{imm[0], imm[1], imm[2]}}; r.dim = 3; break;
    case DK_X: {
        uint64_t ex = i << (TW_MAX_LOG - e.logomega);
        r.v.v[0] = gl_mul(e.x_start, gl_mul(e.tw_lo[ex & (TW_LEVEL_SIZE - 1)], e.tw_hi[ex >> TW_LEVEL_BITS]));
        break;
    }
    case DK_I3: r.v = gl3{{gload(ptr + 3 * i), gload(ptr + 3 * i + 1), gload(ptr + 3 * i + 2)}}; r.dim = 3; break;
    case DK_ZI: r.v.v[0] = gload(ptr + (i & (uint32_t)ii)); break;
    default: break;
    }
    return r;
}

// One wave per workgroup, one row per lane.  Instruction k is one pre-decoded
// 128-byte ZOp record read with scalar loads; operands, op and destination
// are all wave-uniform branches.
__global__ void __launch_bounds__(ZXP_THREADS) k_zxp_eval(ZxpEnv e)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t zlds[];
    const int lane = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * ZXP_THREADS + lane;
    const uint64_t dom = 1ULL << e.logdom;
    const bool active = i < dom;
    const uint64_t ir = active ? i : 0;
    const uint64_t dmask = e.rmask;
    for (uint32_t k = 0; k < e.n_instr; k++) {
        const ZOp &z = e.prog[k];
        const uint32_t op = z.op;
        Val r;
        if (op >= ZXP_DOT1) {
            // linear combination (csrc/zxp_compile.cpp): sum of coef * source,
            // carry-free limb accumulation, one reduction per component
            const uint32_t *k0 = reinterpret_cast<const uint32_t *>(z.ima);
            Dot3 d0(k0), d1(k0 + 3), d2(k0 + 6);
            const ZTerm *T = e.terms + z.ia;
            const int nt = z.ib;
            if (op == ZXP_DOT3) {
                for (int t = 0; t < nt; t++) {
                    const ZTerm &tt = T[t];
                    const uint64_t a =
                        tt.kind == DK_T1 ? zlds[tt.ii + lane] : tt.ptr[(ir + (uint64_t)(int64_t)tt.ii) & dmask];
                    d0.term(a, tt.c[0]);
                    d1.term(a, tt.c[1]);
                    d2.term(a, tt.c[2]);
                }
                r.v = gl3{{d0.fin(), d1.fin(), d2.fin()}};
                r.dim = 3;
            } else {
                for (int t = 0; t < nt; t++) {
                    const ZTerm &tt = T[t];
                    const uint64_t a =
                        tt.kind == DK_T1 ? zlds[tt.ii + lane] : tt.ptr[(ir + (uint64_t)(int64_t)tt.ii) & dmask];
                    d0.term(a, tt.c[0]);
                }
                r.v = gl3{{d0.fin(), 0, 0}};
                r.dim = 1;
            }
        } else {
        Val a = zxp_load(e, z.ka, z.pa, z.ia, z.lda, z.ima, zlds, lane, ir);
        if (op == ZXP_COPY) {
            r = a;
        } else {
            Val b = zxp_load(e, z.kb, z.pb, z.ib, z.ldb, z.imb, zlds, lane, ir);
            r.dim = (a.dim == 3 || b.dim == 3) ? 3 : 1;
            r.v.v[1] = r.v.v[2] = 0;
            if (op == ZXP_MUL) {
                if (a.dim == 3 && b.dim == 3)
                    r.v = gl3_mul(a.v, b.v);
                else if (a.dim == 3)
                    r.v = gl3_mul1(a.v, b.v.v[0]);
                else if (b.dim == 3)
                    r.v = gl3_mul1(b.v, a.v.v[0]);
                else
                    r.v = gl3{{gl_mul(a.v.v[0], b.v.v[0]), 0, 0}};
            } else if (op == ZXP_ADD) {
                if (r.dim == 3)
                    r.v = gl3_add(a.v, b.v);  // a base operand carries zeros in components 1, 2
                else
                    r.v.v[0] = gl_add(a.v.v[0], b.v.v[0]);
            } else {
                if (r.dim == 3)
                    r.v = gl3_sub(a.v, b.v);
                else
                    r.v.v[0] = gl_sub(a.v.v[0], b.v.v[0]);
            }
        }
        }
        switch (z.kd) {
        case DK_T1: zlds[z.id + lane] = r.v.v[0]; break;
        case DK_T3: {
            uint64_t *p = zlds + z.id + lane;
            p[0] = r.v.v[0];
            p[ZXP_THREADS] = r.dim == 3 ? r.v.v[1] : 0;
            p[2 * ZXP_THREADS] = r.dim == 3 ? r.v.v[2] : 0;
            break;
        }
        case DK_C1:
        case DK_C3:
            if (active) {
                uint64_t *p = z.pd + ((i + (uint64_t)(int64_t)z.id) & e.rmask);
                p[0] = gl_canon(r.v.v[0]);
                if (z.kd == DK_C3) {
                    p[z.ldd] = r.dim == 3 ? gl_canon(r.v.v[1]) : 0;
                    p[2 * (uint64_t)z.ldd] = r.dim == 3 ? gl_canon(r.v.v[2]) : 0;
                }
            }
            break;
        default: break;
        }
    }
}

// ---------------------------------------------------------------- calculateZ
// Z[k] = prod_{i<k} num[i] / den[i]  (starks.cpp:146-224, polinomial.hpp:560-607).
// Tiles of Z_TILE = 256 x 8 rows.  Global traffic is always row-coalesced (lane
// = consecutive row); the per-thread CONTIGUOUS runs a prefix product needs are
// read from an LDS image of the tile.
//   k_z_ratio:  ratio = num / den (Montgomery batch inversion over each
//               thread's 8 strided rows), LDS image, per-thread run products,
//               block scan -> per-thread exclusive prefixes + tile total
//   k_z_totals: exclusive prefix of the tile totals (one workgroup)
//   k_z_apply:  z = tile prefix * thread prefix * running product, through LDS
constexpr int BI_CHUNK = 16;  // k_xdiv_rows / k_ext: rows per thread sharing one inversion
constexpr int SCAN_THREADS = 256;
constexpr int Z_PER = 4;
constexpr uint64_t Z_TILE = SCAN_THREADS * Z_PER;
// LDS slot of tile row e: one pad slot per Z_PER rows (run reads: 2-way bank conflicts)
__device__ __forceinline__ int z_slot(int e) { return e + e / Z_PER; }
constexpr int Z_SLOTS = Z_TILE + Z_TILE / Z_PER;

__device__ gl3 block_exclusive_scan3(gl3 v, gl3 *sh, gl3 *total)
{
    // Hillis-Steele inclusive scan over 256 threads in LDS, then shift
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int off = 1; off < SCAN_THREADS; off <<= 1) {
        gl3 x = sh[t];
        gl3 y = t >= off ? sh[t - off] : gl3{{1, 0, 0}};
        __syncthreads();
        sh[t] = t >= off ? gl3_mul(x, y) : x;
        __syncthreads();
    }
    gl3 excl = t ? sh[t - 1] : gl3{{1, 0, 0}};
    *total = sh[SCAN_THREADS - 1];
    __syncthreads();
    return excl;
}

__device__ __forceinline__ void lds_st3(uint64_t *img, int slot, const gl3 &v)
{
    img[slot] = v.v[0];
    img[Z_SLOTS + slot] = v.v[1];
    img[2 * Z_SLOTS + slot] = v.v[2];
}
__device__ __forceinline__ gl3 lds_ld3(const uint64_t *img, int slot)
{
    return gl3{{img[slot], img[Z_SLOTS + slot], img[2 * Z_SLOTS + slot]}};
}

__global__ void __launch_bounds__(SCAN_THREADS) k_z_ratio(uint64_t *ratio, uint64_t *thr_pre, uint64_t *tile_tot,
                                                          const uint64_t *num, uint64_t num_ld, const uint64_t *den,
                                                          uint64_t den_ld, uint64_t n)
{
    __shared__ uint64_t img[3 * Z_SLOTS];
    __shared__ gl3 sh[SCAN_THREADS];
    const int t = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * Z_TILE;
    gl3 pre[Z_PER];
    gl3 acc{{1, 0, 0}};
#pragma unroll
    for (int j = 0; j < Z_PER; j++) {
        const uint64_t k = base + j * SCAN_THREADS + t;
        const gl3 d = k < n ? ld3(den + k, den_ld) : gl3{{1, 0, 0}};
        acc = j ? gl3_mul(acc, d) : d;
        pre[j] = acc;
    }
    gl3 inv = gl3_inv(acc);
#pragma unroll
    for (int jj = 0; jj < Z_PER; jj++) {
        const int j = Z_PER - 1 - jj;
        const int e = j * SCAN_THREADS + t;
        const uint64_t k = base + e;
        const gl3 dinv = j ? gl3_mul(inv, pre[j - 1]) : inv;
        gl3 r{{1, 0, 0}};
        if (k < n) {
            r = gl3_mul(ld3(num + k, num_ld), dinv);
            uint64_t *o = ratio + 3 * k;
            o[0] = r.v[0];
            o[1] = r.v[1];
            o[2] = r.v[2];
            if (j) inv = gl3_mul(inv, ld3(den + k, den_ld));
        }
        lds_st3(img, z_slot(e), r);
    }
    __syncthreads();
    gl3 run = lds_ld3(img, z_slot(t * Z_PER));
#pragma unroll
    for (int i = 1; i < Z_PER; i++) run = gl3_mul(run, lds_ld3(img, z_slot(t * Z_PER + i)));
    gl3 tot;
    const gl3 ex = block_exclusive_scan3(run, sh, &tot);
    uint64_t *tp = thr_pre + 3 * ((uint64_t)blockIdx.x * SCAN_THREADS + t);
    tp[0] = ex.v[0];
    tp[1] = ex.v[1];
    tp[2] = ex.v[2];
    if (t == 0) {
        tile_tot[3 * blockIdx.x] = tot.v[0];
        tile_tot[3 * blockIdx.x + 1] = tot.v[1];
        tile_tot[3 * blockIdx.x + 2] = tot.v[2];
    }
}

// exclusive prefix of the tile totals times z0: each thread multiplies a
// contiguous run of ceil(ntiles / 256) totals, one block scan, then the run is
// re-walked; *total = z0 * prod of all ratios (the closing value)
__global__ void __launch_bounds__(SCAN_THREADS) k_z_totals(uint64_t *tile_pre, const uint64_t *tile_tot,
                                                           uint64_t ntiles, gl3 z0, uint64_t *total)
{
    __shared__ gl3 sh[SCAN_THREADS];
    const uint64_t per = (ntiles + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint64_t b0 = threadIdx.x * per;
    uint64_t b1 = b0 + per;
    if (b1 > ntiles) b1 = ntiles;
    gl3 acc{{1, 0, 0}};
    for (uint64_t b = b0; b < b1; b++) acc = gl3_mul(acc, ld3(tile_tot + 3 * b, 1));
    gl3 tot;
    gl3 run = gl3_mul(z0, block_exclusive_scan3(acc, sh, &tot));
    for (uint64_t b = b0; b < b1; b++) {
        tile_pre[3 * b] = run.v[0];
        tile_pre[3 * b + 1] = run.v[1];
        tile_pre[3 * b + 2] = run.v[2];
        run = gl3_mul(run, ld3(tile_tot + 3 * b, 1));
    }
    if (threadIdx.x == 0) {
        const gl3 t = gl3_canon(gl3_mul(z0, tot));
        total[0] = t.v[0];
        total[1] = t.v[1];
        total[2] = t.v[2];
    }
}

__global__ void __launch_bounds__(SCAN_THREADS) k_z_apply(uint64_t *z, uint64_t z_ld, const uint64_t *ratio,
                                                          const uint64_t *thr_pre, const uint64_t *tile_pre,
                                                          uint64_t n)
{
    __shared__ uint64_t img[3 * Z_SLOTS];
    const int t = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * Z_TILE;
#pragma unroll
    for (int j = 0; j < Z_PER; j++) {
        const int e = j * SCAN_THREADS + t;
        const uint64_t k = base + e;
        lds_st3(img, z_slot(e), k < n ? ld3(ratio + 3 * k, 1) : gl3{{1, 0, 0}});
    }
    gl3 run = gl3_mul(ld3(tile_pre + 3 * blockIdx.x, 1), ld3(thr_pre + 3 * ((uint64_t)blockIdx.x * SCAN_THREADS + t), 1));
    __syncthreads();
#pragma unroll
    for (int i = 0; i < Z_PER; i++) {  // exclusive: z[k] = prod_{i<k} ratio[i]
        const int sl = z_slot(t * Z_PER + i);
        const gl3 r = lds_ld3(img, sl);
        lds_st3(img, sl, run);
        run = gl3_mul(run, r);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < Z_PER; j++) {
        const int e = j * SCAN_THREADS + t;
        const uint64_t k = base + e;
        if (k < n) st3(z + k, z_ld, lds_ld3(img, z_slot(e)));
    }
}

// ---------------------------------------------------------------- evmap
constexpr int EV_THREADS = 256;

// Sub-entry form: an F_p^3 entry pol = p0 + p1 X + p2 X^2 is three base
// sub-entries, S_j = sum_k L(k) p_j[k] and pol(xi) = S_0 + S_1 X + S_2 X^2
// (k_evmap_sum_subs).  EV_G sub-entries with the same L (prime or not) form
// a group: each thread turns L(k) into Dot3 limbs once per row, and every
// sub-entry's term costs 6 carry-free multiply-adds per component, instead of
// a reduced F_p^3 product per entry and row.
constexpr int EV_G = 8;  // group slots; a launch uses the first G (template)
constexpr uint64_t EV_ROWS_PER_THREAD = 240;  // Dot3 accumulators: < 2^63 for <= 250 terms
struct EvGroup {
    const uint64_t *col[EV_G];  // null: unused slot
    uint32_t prime, sub0;
};

// U rows per thread and iteration: all their loads are issued before the
// multiply-adds (memory-level parallelism at the kernel's modest occupancy).
template <int G, int U>
__global__ void __launch_bounds__(EV_THREADS) k_evmap_groups(uint64_t *partial, const EvGroup *groups,
                                                            const uint64_t *lev, const uint64_t *lpev, uint64_t l_ld,
                                                            uint64_t n, uint32_t eb, uint64_t rows_per_block)
{
    __shared__ gl3 sh[EV_THREADS];
    const EvGroup g = groups[blockIdx.x];
    const uint64_t blk = blockIdx.y;
    const uint64_t *L = g.prime ? lpev : lev;
    Dot3 acc[G][3];
    const uint64_t r0 = blk * rows_per_block;
    uint64_t r1 = r0 + rows_per_block;
    if (r1 > n) r1 = n;
    for (uint64_t k0 = r0 + threadIdx.x; k0 < r1; k0 += (uint64_t)EV_THREADS * U) {
        gl3 c[U];
        uint64_t a[U][G];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = k0 + (uint64_t)u * EV_THREADS;
            const bool in = k < r1;  // out of range: zero terms (still within the 240-term bound)
            c[u] = in ? ld3(L + k, l_ld) : gl3{{0, 0, 0}};
#pragma unroll
            for (int e = 0; e < G; e++) a[u][e] = (in && g.col[e]) ? gload(g.col[e] + (k << eb)) : 0;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t cl[3][6];
#pragma unroll
            for (int j = 0; j < 3; j++) Dot3::limbs(c[u].v[j], cl[j]);
#pragma unroll
            for (int e = 0; e < G; e++) {
#pragma unroll
                for (int j = 0; j < 3; j++) acc[e][j].term(a[u][e], cl[j]);
            }
        }
    }
#pragma unroll
    for (int e = 0; e < G; e++) {
        if (!g.col[e]) break;
        sh[threadIdx.x] = gl3{{acc[e][0].fin(), acc[e][1].fin(), acc[e][2].fin()}};
        __syncthreads();
        for (int off = EV_THREADS / 2; off > 0; off >>= 1) {
            if (threadIdx.x < off) sh[threadIdx.x] = gl3_add(sh[threadIdx.x], sh[threadIdx.x + off]);
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            uint64_t *o = partial + 3 * ((uint64_t)(g.sub0 + e) * gridDim.y + blk);
            o[0] = sh[0].v[0];
            o[1] = sh[0].v[1];
            o[2] = sh[0].v[2];
        }
        __syncthreads();
    }
}

// evals[e] = sum_j X^j * (sum over blocks of sub-entry j's partials); subs: 3 per entry, -1 = none
__global__ void k_evmap_sum_subs(uint64_t *evals, const uint64_t *partial, const int32_t *subs, uint32_t n_ev,
                                 uint32_t nblk)
{
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_ev) return;
    gl3 acc{{0, 0, 0}};
    for (int j = 2; j >= 0; j--) {  // Horner in X; x^3 = x + 1: (a0 + a1 x + a2 x^2) x = a2 + (a0 + a2) x + a1 x^2
        acc = gl3{{acc.v[2], gl_add(acc.v[0], acc.v[2]), acc.v[1]}};
        const int32_t sub = subs[3 * e + j];
        if (sub < 0) continue;
        for (uint32_t b = 0; b < nblk; b++) {
            const uint64_t *p = partial + 3 * ((uint64_t)sub * nblk + b);
            acc = gl3_add(acc, gl3{{p[0], p[1], p[2]}});
        }
    }
    acc = gl3_canon(acc);
    evals[3 * e] = acc.v[0];
    evals[3 * e + 1] = acc.v[1];
    evals[3 * e + 2] = acc.v[2];
}

// ---------------------------------------------------------------- xDivXSub
// xdiv[k] = x_k / (x_k - xi), xdivw[k] = x_k / (x_k - w xi), x_k = 7 * omega_2n^k
// out_w[k] = scale * x_k / (x_k - a_w), x_k = shift * omega_{2^logn}^(row0 + k),
// k < nrows, w = 0, 1; BI_CHUNK rows per thread share one F_p^3 inversion.
// interleaved (scale 1): out_w + 3 k + c (the xDivXSub layout), else out_w + c ld + k.
// xDivXSubXi / WXi (starks.cpp:344-366): shift 7 on the extended domain,
// scale 1.  LEv / LpEv (starks.cpp:308-324, INTT of the powers of xi and
// w xi): with x_k = w_N^k, (1/N) sum_j xi^j w^-jk = ((1 - xi^N) / N) x_k /
// (x_k - xi), the same field value row by row.
template <bool INTERLEAVED>
__global__ void __launch_bounds__(256) k_xdiv_rows(uint64_t *out0, uint64_t *out1, uint64_t ld, gl3 a0, gl3 a1,
                                                   uint64_t shift, gl3 scale, uint32_t logn, uint64_t row0,
                                                   uint64_t nrows, const uint64_t *tw_lo, const uint64_t *tw_hi)
{
    const uint64_t n = 1ULL << logn;
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int which = 0; which < 2; which++) {
        const gl3 s = which ? a1 : a0;
        uint64_t *out = which ? out1 : out0;
        gl3 pre[BI_CHUNK];
        uint64_t xs[BI_CHUNK];
        gl3 acc{{1, 0, 0}};
#pragma unroll
        for (int j = 0; j < BI_CHUNK; j++) {
            uint64_t k = t + j * T;
            uint64_t ex = ((row0 + k) & (n - 1)) << (TW_MAX_LOG - logn);
            xs[j] = gl_mul(shift, gl_mul(tw_lo[ex & (TW_LEVEL_SIZE - 1)], tw_hi[ex >> TW_LEVEL_BITS]));
            gl3 d = k < nrows ? gl3{{gl_sub(xs[j], s.v[0]), gl_neg(s.v[1]), gl_neg(s.v[2])}} : gl3{{1, 0, 0}};
            acc = j ? gl3_mul(acc, d) : d;
            pre[j] = acc;
        }
        gl3 inv = gl3_inv(acc);
#pragma unroll
        for (int jj = 0; jj < BI_CHUNK; jj++) {  // (descending j; this form unrolls, keeping pre[] in registers)
            const int j = BI_CHUNK - 1 - jj;
            uint64_t k = t + j * T;
            gl3 dinv = j ? gl3_mul(inv, pre[j - 1]) : inv;
            if (k < nrows) {
                gl3 d{{gl_sub(xs[j], s.v[0]), gl_neg(s.v[1]), gl_neg(s.v[2])}};
                gl3 r = gl3_mul1(dinv, xs[j]);
                if constexpr (!INTERLEAVED) r = gl3_mul(r, scale);  // (xDivXSub: scale 1)
                r = gl3_canon(r);
                if constexpr (INTERLEAVED) {
                    out[3 * k] = r.v[0];
                    out[3 * k + 1] = r.v[1];
                    out[3 * k + 2] = r.v[2];
                } else {
                    out[k] = r.v[0];
                    out[ld + k] = r.v[1];
                    out[2 * ld + k] = r.v[2];
                }
                inv = gl3_mul(inv, d);
            }
        }
    }
}

// ---------------------------------------------------------------- powers & split
// out column-major (3 columns, ld): out[k] = base^k, k < n.  Thread t of T
// owns rows t + j*T (coalesced stores): r = base^t, stepped by base^T
__device__ __forceinline__ gl3 gl3_pow(gl3 b, uint64_t e)
{
    gl3 r{{1, 0, 0}};
    while (e) {
        if (e & 1) r = gl3_mul(r, b);
        b = gl3_mul(b, b);
        e >>= 1;
    }
    return r;
}

__global__ void k_ext_powers(uint64_t *out, uint64_t ld, gl3 base, uint64_t n)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    if (t >= n) return;
    gl3 r = gl3_pow(base, t);
    const gl3 step = gl3_pow(base, T);
    for (uint64_t k = t; k < n; k += T) {
        st3(out + k, ld, r);
        r = gl3_mul(r, step);
    }
}

// cols[c][k] *= base^k, k < n: thread t owns rows t + j*T (coalesced), its
// factor starts at base^t and steps by base^T
__global__ void k_scale_powers(uint64_t *cols, uint64_t ld, uint32_t ncols, uint64_t n, uint64_t base, uint64_t base_t,
                               uint32_t per)
{
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t f = gl_pow(base, t);
    for (uint32_t j = 0; j < per; j++) {
        const uint64_t k = t + (uint64_t)j * T;
        if (k >= n) break;
        for (uint32_t c = 0; c < ncols; c++) cols[(uint64_t)c * ld + k] = gl_canon(gl_mul(cols[(uint64_t)c * ld + k], f));
        f = gl_mul(f, base_t);
    }
}

// qq2 column stride*p+d, row k < N: qq1_d[p N + k] * shiftIn^p, d < dim
// (starks.cpp:266-281: dim = stride = 3; the row-sharded prover's column
// owners split one column, dim 1, into every third output column)
__global__ void k_qsplit(uint64_t *qq2, uint64_t ld2, const uint64_t *qq1, uint64_t ld1, uint64_t n, uint32_t qdeg,
                         uint64_t shift_in, uint32_t dim, uint32_t stride)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint64_t f = 1;
    for (uint32_t p = 0; p < qdeg; p++) {
        for (uint32_t d = 0; d < dim; d++)
            qq2[(uint64_t)(stride * p + d) * ld2 + k] =
                gl_canon(gl_mul(qq1[(uint64_t)d * ld1 + (uint64_t)p * n + k], f));
        f = gl_mul(f, shift_in);
    }
}

// interleave 3 column-major ext columns into an interleaved (n x 3) array
__global__ void k_cols3_to_interleaved(uint64_t *out, const uint64_t *cols, uint64_t ld, uint64_t n)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    out[3 * k] = cols[k];
    out[3 * k + 1] = cols[ld + k];
    out[3 * k + 2] = cols[2 * ld + k];
}

// ---------------------------------------------------------------- host side
static inline uint32_t nblk(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

int rand_cols(uint64_t *base, uint64_t ld, const uint32_t *cols_dev, uint32_t ncols, uint64_t nrows, uint64_t seed,
              uint64_t stream, uint64_t row0, uint64_t rmask, hipStream_t s)
{
    if (!ncols || !nrows) return 0;
    hipLaunchKernelGGL(k_rand_cols, dim3(nblk(nrows, 256), ncols), dim3(256), 0, s, base, ld, cols_dev, ncols, nrows,
                       seed, stream, row0, rmask);
    return check_launch("k_rand_cols");
}

int copy_rows(uint64_t *dst, uint64_t dld, uint64_t drow0, const uint32_t *dcols, const uint64_t *src, uint64_t sld,
              uint64_t srow0, uint64_t smask, const uint32_t *scols, uint32_t ncols, uint64_t nrows, hipStream_t s)
{
    if (!ncols || !nrows) return 0;
    hipLaunchKernelGGL(k_copy_rows, dim3(nblk(nrows, 256), ncols), dim3(256), 0, s, dst, dld, drow0, dcols, src, sld,
                       srow0, smask, scols, ncols, nrows);
    return check_launch("k_copy_rows");
}

int zxp_eval(const ZxpLaunch &L, hipStream_t s)
{
    Ctx &c = ctx();
    ZxpEnv e;
    e.prog = L.prog;
    e.terms = L.terms;
    e.n_instr = L.n_instr;
    e.logdom = L.logdom;
    e.logomega = L.logomega;
    e.rmask = L.wrap ? (1ULL << L.logdom) - 1 : ~0ULL;
    e.x_start = L.x_start;
    e.tw_lo = c.tw_lo[0];
    e.tw_hi = c.tw_hi[0];
    const uint64_t slots = (uint64_t)L.n_tmp1 + 3ULL * L.n_tmp3;
    size_t lds = (size_t)(slots ? slots : 1) * ZXP_THREADS * sizeof(uint64_t);
    if (lds > 160 * 1024) return set_error(ZKGPU_ERR_ARG, "zxp: %llu temp slots exceed LDS", (unsigned long long)slots);
    const uint64_t dom = 1ULL << L.logdom;
    prof_begin(s);
    hipLaunchKernelGGL(k_zxp_eval, dim3(nblk(dom, ZXP_THREADS)), dim3(ZXP_THREADS), lds, s, e);
    prof_end("k_zxp_eval", L.bytes, s);
    return check_launch("k_zxp_eval");
}

size_t calculate_z_scratch_words(uint64_t n)
{
    const uint64_t nt = (n + Z_TILE - 1) / Z_TILE;
    return 3 * n + 3 * nt * SCAN_THREADS + 6 * nt + 4;
}

int calculate_z(uint64_t *z, uint64_t z_ld, const uint64_t *num, uint64_t num_ld, const uint64_t *den,
                uint64_t den_ld, uint64_t n, const uint64_t z0[3], uint64_t *scratch, uint64_t *total_dev, hipStream_t s)
{
    // scratch: ratio (3n) + per-thread prefixes (3 * 256 per tile) + tile totals + tile prefixes
    const uint64_t nt = (n + Z_TILE - 1) / Z_TILE;
    uint64_t *ratio = scratch;
    uint64_t *thr = ratio + 3 * n;
    uint64_t *tot = thr + 3 * nt * SCAN_THREADS;
    uint64_t *pre = tot + 3 * nt;
    prof_begin(s);
    hipLaunchKernelGGL(k_z_ratio, dim3((uint32_t)nt), dim3(SCAN_THREADS), 0, s, ratio, thr, tot, num, num_ld, den,
                       den_ld, n);
    prof_end("k_z_ratio", 8.0 * 9 * n, s);
    const gl3 z0v{{z0[0], z0[1], z0[2]}};
    hipLaunchKernelGGL(k_z_totals, dim3(1), dim3(SCAN_THREADS), 0, s, pre, tot, nt, z0v, total_dev);
    prof_begin(s);
    hipLaunchKernelGGL(k_z_apply, dim3((uint32_t)nt), dim3(SCAN_THREADS), 0, s, z, z_ld, ratio, thr, pre, n);
    prof_end("k_z_apply", 8.0 * 6 * n, s);
    return check_launch("calculateZ");
}

size_t evmap_group_size() { return sizeof(EvGroup); }
uint32_t evmap_group_width() { return EV_G; }
uint64_t evmap_rows_per_block() { return EV_ROWS_PER_THREAD * EV_THREADS; }

int evmap_groups(uint64_t *evals, const void *groups_dev, uint32_t n_groups, uint32_t width, uint32_t unroll,
                 const int32_t *subs_dev,
                 uint32_t n_ev, uint32_t n_sub, const uint64_t *lev, const uint64_t *lpev, uint64_t l_ld, uint64_t n,
                 uint32_t eb, uint64_t *partial, hipStream_t s)
{
    if (!n_ev) return 0;
    const uint64_t rpb = evmap_rows_per_block();
    const uint32_t nblk_ = (uint32_t)((n + rpb - 1) / rpb);
    const EvGroup *g = (const EvGroup *)groups_dev;
    const dim3 grid(n_groups, nblk_);
    prof_begin(s);
#define EVG(G_, U_)                                                                                                  \
    case G_ * 16 + U_:                                                                                                 \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_evmap_groups<G_, U_>), grid, dim3(EV_THREADS), 0, s, partial, g, lev,      \
                           lpev, l_ld, n, eb, rpb);                                                                    \
        break;
    switch (width * 16 + unroll) {
        EVG(1, 1) EVG(1, 2) EVG(1, 4) EVG(2, 1) EVG(2, 2) EVG(2, 4) EVG(4, 1) EVG(4, 2) EVG(4, 4)
    default: return set_error(ZKGPU_ERR_ARG, "evmap group width %u unroll %u", width, unroll);
    }
#undef EVG
    prof_end("k_evmap", 8.0 * n * n_sub + 24.0 * n * 2, s);
    hipLaunchKernelGGL(k_evmap_sum_subs, dim3(nblk(n_ev, 64)), dim3(64), 0, s, evals, partial, subs_dev, n_ev, nblk_);
    return check_launch("k_evmap_groups");
}

static gl3 h_gl3(const uint64_t v[3]) { return gl3{{v[0] % ZK_P, v[1] % ZK_P, v[2] % ZK_P}}; }

int xdiv_rows(uint64_t *out0, uint64_t *out1, uint64_t ld, int interleaved, const uint64_t a0[3],
              const uint64_t a1[3], uint64_t shift, const uint64_t scale[3], uint32_t logn, uint64_t row0,
              uint64_t nrows, hipStream_t s)
{
    if (!nrows) return 0;
    Ctx &c = ctx();
    const uint64_t threads = (nrows + BI_CHUNK - 1) / BI_CHUNK;
    prof_begin(s);
    const gl3 sc = h_gl3(scale);
    if (interleaved && !(sc.v[0] == 1 && sc.v[1] == 0 && sc.v[2] == 0))
        return set_error(ZKGPU_ERR_ARG, "xdiv_rows: the interleaved form has scale 1");
    if (interleaved)
        hipLaunchKernelGGL(k_xdiv_rows<true>, dim3(nblk(threads, 256)), dim3(256), 0, s, out0, out1, ld, h_gl3(a0),
                           h_gl3(a1), shift, sc, logn, row0, nrows, c.tw_lo[0], c.tw_hi[0]);
    else
        hipLaunchKernelGGL(k_xdiv_rows<false>, dim3(nblk(threads, 256)), dim3(256), 0, s, out0, out1, ld, h_gl3(a0),
                           h_gl3(a1), shift, sc, logn, row0, nrows, c.tw_lo[0], c.tw_hi[0]);
    prof_end("k_xdiv_rows", 48.0 * nrows, s);
    return check_launch("k_xdiv_rows");
}

int xdivxsub(uint64_t *xdiv, uint64_t *xdivw, const uint64_t xi[3], uint64_t w, uint32_t logn, hipStream_t s)
{
    return xdivxsub_rows(xdiv, xdivw, xi, w, logn, 0, 1ULL << logn, s);
}

int xdivxsub_rows(uint64_t *xdiv, uint64_t *xdivw, const uint64_t xi[3], uint64_t w, uint32_t logn, uint64_t row0,
                  uint64_t nrows, hipStream_t s)
{
    const uint64_t wx[3] = {h_mul(xi[0] % ZK_P, w), h_mul(xi[1] % ZK_P, w), h_mul(xi[2] % ZK_P, w)};
    const uint64_t one[3] = {1, 0, 0};
    return xdiv_rows(xdiv + 3 * row0, xdivw + 3 * row0, 0, 1, xi, wx, 7, one, logn, row0, nrows, s);
}

int ext_powers(uint64_t *out, uint64_t ld, const uint64_t base[3], uint64_t n, hipStream_t s)
{
    gl3 b{{base[0] % ZK_P, base[1] % ZK_P, base[2] % ZK_P}};
    const uint32_t per = 64;
    const uint64_t threads = (n + per - 1) / per;
    hipLaunchKernelGGL(k_ext_powers, dim3(nblk(threads, 256)), dim3(256), 0, s, out, ld, b, n);
    return check_launch("k_ext_powers");
}

int scale_powers(uint64_t *cols, uint64_t ld, uint32_t ncols, uint64_t n, uint64_t base, hipStream_t s)
{
    const uint32_t per = 64;
    const uint64_t threads = (n + per - 1) / per;
    const uint32_t blocks = nblk(threads, 256);
    const uint64_t T = (uint64_t)blocks * 256;
    hipLaunchKernelGGL(k_scale_powers, dim3(blocks), dim3(256), 0, s, cols, ld, ncols, n, base % ZK_P,
                       h_pow(base, T), per);
    return check_launch("k_scale_powers");
}

int qsplit(uint64_t *qq2, uint64_t ld2, const uint64_t *qq1, uint64_t ld1, uint64_t n, uint32_t qdeg,
           uint64_t shift_in, uint32_t dim, uint32_t stride, hipStream_t s)
{
    hipLaunchKernelGGL(k_qsplit, dim3(nblk(n, 256)), dim3(256), 0, s, qq2, ld2, qq1, ld1, n, qdeg, shift_in, dim,
                       stride);
    return check_launch("k_qsplit");
}

int cols3_to_interleaved(uint64_t *out, const uint64_t *cols, uint64_t ld, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_cols3_to_interleaved, dim3(nblk(n, 256)), dim3(256), 0, s, out, cols, ld, n);
    return check_launch("k_cols3_to_interleaved");
}

}  // namespace zk
