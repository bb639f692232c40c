// Poseidon-GL permutation, linear hash and Merkle tree kernels for gfx950.
//
// Replaces PoseidonGoldilocks::{hash_full_result, hash, linear_hash,
// merkletree_avx} (submodule, absent; call sites merkleTreeGL.cpp:37-44,
// transcript.cpp:23,46, build_const_tree.cpp:582) and MerkleTreeGL's
// getGroupProof (merkleTreeGL.cpp:12-35).
//
// Permutation: poseidon_perm.hpp (perm_fast) -- bit-identical to the
// reference's form at poseidon_g_executor.cpp:201-231 / .hpp:29-51, evaluated
// with folded round constants and the partial rounds as block dot products.
// Integer VALU-bound: one thread per permutation, the 12-lane state in VGPRs,
// table coefficients as wave-uniform scalar loads.
//
// Leaves: one thread per row; a column-major (SoA) source makes each of the
// ceil(ncols/8) absorption steps a fully coalesced 8-column read.
#include "poseidon_perm.hpp"
#include "zkgpu_internal.hpp"

namespace zk {

// ---------------------------------------------------------------- kernels
__global__ void k_poseidon_batch(uint64_t *out, const uint64_t *in, uint64_t n, int full)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t st[12];
#pragma unroll
    for (int k = 0; k < 12; k++) st[k] = in[i * 12 + k];
    poseidon_perm(st);
    const int w = full ? 12 : 4;
    for (int k = 0; k < w; k++) out[i * w + k] = gl_canon(st[k]);
}

// leaf digests from a column-major source (column c at src + c*ld); SPLIT:
// columns from `split` on (a multiple of 8, so no absorption chunk straddles
// it) at src2 + (c - split)*ld -- one section held in two regions (the lean
// plan's stage-1 commit, host/starks.cpp)
template <bool SPLIT>
__device__ __forceinline__ void leaves_cols(uint64_t *digests, const uint64_t *__restrict__ src, uint64_t ncols,
                                            uint64_t nrows, uint64_t ld, const uint64_t *__restrict__ src2,
                                            uint64_t split)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    uint64_t st[12];
    if (ncols <= 4) {
#pragma unroll
        for (int k = 0; k < 4; k++) st[k] = (uint64_t)k < ncols ? src[k * ld + i] : 0;
    } else {
#pragma unroll
        for (int k = 0; k < 12; k++) st[k] = 0;
        for (uint64_t c0 = 0; c0 < ncols; c0 += 8) {
            uint64_t nk = ncols - c0 < 8 ? ncols - c0 : 8;
            if (c0) {
#pragma unroll
                for (int k = 0; k < 4; k++) st[8 + k] = st[k];
            }
            const uint64_t *b = (!SPLIT || c0 < split) ? src + c0 * ld : src2 + (c0 - split) * ld;
#pragma unroll
            for (int k = 0; k < 8; k++) st[k] = (uint64_t)k < nk ? b[k * ld + i] : 0;
            poseidon_perm(st);
        }
    }
    uint64_t *d = digests + 4 * i;
#pragma unroll
    for (int k = 0; k < 4; k++) d[k] = ncols <= 4 ? st[k] : gl_canon(st[k]);
}
__global__ void __launch_bounds__(256) k_leaves_cols(uint64_t *digests, const uint64_t *__restrict__ src,
                                                    uint64_t ncols, uint64_t nrows, uint64_t ld)
{
    leaves_cols<false>(digests, src, ncols, nrows, ld, nullptr, ncols);
}
__global__ void __launch_bounds__(256) k_leaves_cols2(uint64_t *digests, const uint64_t *__restrict__ src,
                                                     uint64_t ncols, uint64_t nrows, uint64_t ld,
                                                     const uint64_t *__restrict__ src2, uint64_t split)
{
    leaves_cols<true>(digests, src, ncols, nrows, ld, src2, split);
}

// leaf digests from a row-major source (row i at src + i*ncols)
__global__ void __launch_bounds__(256) k_leaves_rows(uint64_t *digests, const uint64_t *__restrict__ src,
                                                    uint64_t ncols, uint64_t nrows)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    const uint64_t *row = src + i * ncols;
    uint64_t st[12];
    if (ncols <= 4) {
#pragma unroll
        for (int k = 0; k < 4; k++) st[k] = (uint64_t)k < ncols ? row[k] : 0;
    } else {
#pragma unroll
        for (int k = 0; k < 12; k++) st[k] = 0;
        for (uint64_t c0 = 0; c0 < ncols; c0 += 8) {
            uint64_t nk = ncols - c0 < 8 ? ncols - c0 : 8;
            if (c0) {
#pragma unroll
                for (int k = 0; k < 4; k++) st[8 + k] = st[k];
            }
#pragma unroll
            for (int k = 0; k < 8; k++) st[k] = (uint64_t)k < nk ? row[c0 + k] : 0;
            poseidon_perm(st);
        }
    }
    uint64_t *d = digests + 4 * i;
#pragma unroll
    for (int k = 0; k < 4; k++) d[k] = ncols <= 4 ? st[k] : gl_canon(st[k]);
}

// ---------------------------------------------------------------- lane-parallel form
// Tree levels and leaf sets too small to fill the GPU take the LATENCY of one
// thread's ~19 K-instruction permutation chain (~65 us per level, measured).
// Here one permutation is spread over 16 lanes (lane x < 12 holds st[x], 4
// states per wave): the S-boxes run side by side and each lane forms its MDS
// row sum from the state exchanged through LDS -- ~4 K instructions on the
// critical path.  Textbook round structure (poseidon_g_executor.cpp:201-231):
// add constants, S-box (full rounds: all lanes; partial: lane 0), MDS.
constexpr int LP_LANES = 16;
// Crossover: the lane form costs ~3.1x the instructions per permutation
// (3.8 K VALU per 4 states vs 19.4 K per 64), so it wins while a launch is
// latency-bound: up to ~2^15 concurrent permutations on 256 CUs.
constexpr uint64_t LP_MAX_PERMS = 1ULL << 15;

struct LpCtx {
    uint64_t rc[30];  // this lane's round constants
    uint32_t m[12];   // this lane's MDS row
    uint32_t x;       // state element held (>= 12: idle lane)
    uint64_t *xch;    // the state's 16 exchange slots in LDS
};

__device__ __forceinline__ void lp_init(LpCtx &c, uint64_t *lds)
{
    c.x = threadIdx.x & (LP_LANES - 1);
    const uint32_t xx = c.x < 12 ? c.x : 0;
#pragma unroll
    for (int r = 0; r < 30; r++) c.rc[r] = c.x < 12 ? ZKGPU_POSEIDON_RC[r * 12 + xx] : 0;
#pragma unroll
    for (int y = 0; y < 12; y++) c.m[y] = mds_entry((int)xx, y);
    c.xch = lds + (threadIdx.x & ~(LP_LANES - 1));
}

// the 12 state elements as seen by every lane of the state's group
__device__ __forceinline__ void lp_share(const LpCtx &c, uint64_t s, uint64_t v[12])
{
    c.xch[c.x] = s;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int y = 0; y < 12; y++) v[y] = c.xch[y];
    __builtin_amdgcn_wave_barrier();  // reads done before the next round's write
}

template <int r>
__device__ __forceinline__ void lp_round(const LpCtx &c, uint64_t &s)
{
    {
        s = gl_add(s, c.rc[r]);
        if constexpr (r < 4 || r >= 26)
            s = pow7(s);
        else if (c.x == 0)
            s = pow7(s);
        uint64_t v[12];
        lp_share(c, s, v);
        uint64_t sl = 0, sh = 0;
#pragma unroll
        for (int y = 0; y < 12; y++) {
            sl += (uint64_t)(uint32_t)v[y] * c.m[y];
            sh += (uint64_t)(uint32_t)(v[y] >> 32) * c.m[y];
        }
        // value = sl + sh * 2^32 < 2^75
        uint32_t c1, c2;
        const uint32_t mid = __builtin_addc((uint32_t)(sl >> 32), (uint32_t)sh, 0u, &c1);
        const uint32_t h = __builtin_addc((uint32_t)(sh >> 32), 0u, c1, &c2);
        s = gl_reduce96(((uint64_t)mid << 32) | (uint32_t)sl, h);
    }
}

template <int... rs>
__device__ __forceinline__ void lp_rounds(const LpCtx &c, uint64_t &s, std::integer_sequence<int, rs...>)
{
    (lp_round<rs>(c, s), ...);
}

__device__ __forceinline__ uint64_t lp_perm(const LpCtx &c, uint64_t s)
{
    lp_rounds(c, s, std::make_integer_sequence<int, 30>{});
    return s;
}

// one tree level, 16 lanes per node
__global__ void __launch_bounds__(256) k_merkle_level_lp(uint64_t *dst, const uint64_t *lvl, uint64_t next)
{
    __shared__ uint64_t lds[256];
    LpCtx c;
    lp_init(c, lds);
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / LP_LANES;
    if (i >= next) return;  // whole 16-lane groups
    uint64_t s = c.x < 8 ? lvl[8 * i + c.x] : 0;
    s = lp_perm(c, s);
    if (c.x < 4) dst[4 * i + c.x] = gl_canon(s);
}

// A tree's last levels (<= LP_TAIL nodes: one 16-lane group per node in one
// 1024-thread workgroup) in one launch, a workgroup barrier between levels:
// each level still costs one lane-parallel permutation's latency, but not a
// dependent launch's ~10 us (per-dispatch trace: 7 such levels per tree, ~9
// trees per config-4 proof)
constexpr uint64_t LP_TAIL = 64;
__global__ void __launch_bounds__(1024) k_merkle_tail_lp(uint64_t *lvl, uint64_t pending)
{
    __shared__ uint64_t lds[1024];
    LpCtx c;
    lp_init(c, lds);
    const uint64_t i = threadIdx.x / LP_LANES;
    while (pending > 1) {
        const uint64_t next = pending / 2;
        uint64_t *dst = lvl + 4 * pending;
        if (i < next) {  // whole 16-lane groups
            uint64_t s = c.x < 8 ? lvl[8 * i + c.x] : 0;
            s = lp_perm(c, s);
            if (c.x < 4) dst[4 * i + c.x] = gl_canon(s);
        }
        __syncthreads();  // this level's nodes stored before the next level reads them (one workgroup)
        lvl = dst;
        pending = next;
    }
}

// leaf digests (linear_hash) of a row-major source, 16 lanes per row
__global__ void __launch_bounds__(256) k_leaves_rows_lp(uint64_t *digests, const uint64_t *__restrict__ src,
                                                       uint64_t ncols, uint64_t nrows)
{
    __shared__ uint64_t lds[256];
    LpCtx c;
    lp_init(c, lds);
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / LP_LANES;
    if (i >= nrows) return;
    const uint64_t *row = src + i * ncols;
    uint64_t s;
    if (ncols <= 4) {
        s = c.x < ncols ? row[c.x] : 0;  // copied, not hashed (and not canonicalised)
    } else {
        s = 0;
        for (uint64_t c0 = 0; c0 < ncols; c0 += 8) {
            if (c0) {  // capacity = previous output[0..3]
                uint64_t v[12];
                lp_share(c, s, v);
                s = c.x >= 8 && c.x < 12 ? v[c.x - 8] : s;
            }
            if (c.x < 8) s = c0 + c.x < ncols ? row[c0 + c.x] : 0;
            s = lp_perm(c, s);
        }
        s = gl_canon(s);
    }
    if (c.x < 4) digests[4 * i + c.x] = s;
}

// one tree level: dst[i] = hash(lvl[2i] || lvl[2i+1] || 0000)
__global__ void __launch_bounds__(256) k_merkle_level(uint64_t *dst, const uint64_t *lvl, uint64_t next)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= next) return;
    uint64_t st[12];
#pragma unroll
    for (int k = 0; k < 8; k++) st[k] = lvl[8 * i + k];
#pragma unroll
    for (int k = 8; k < 12; k++) st[k] = 0;
    poseidon_perm(st);
#pragma unroll
    for (int k = 0; k < 4; k++) dst[4 * i + k] = gl_canon(st[k]);
}

// openings: vals[q*ncols + c] = src[row*row_stride + c*col_stride]; sibs[q][l][0..3]
__global__ void k_merkle_open(uint64_t *vals, uint64_t *sibs, const uint64_t *nodes, const uint64_t *src,
                              uint64_t ncols, uint64_t nrows, uint64_t row_stride, uint64_t col_stride,
                              const uint64_t *idx, uint64_t nq, uint32_t nlevels)
{
    uint64_t q = blockIdx.x;
    if (q >= nq) return;
    uint64_t row = idx[q];
    for (uint64_t c = threadIdx.x; c < ncols; c += blockDim.x)
        vals[q * ncols + c] = src[row * row_stride + c * col_stride];
    if (threadIdx.x == 0) {
        uint64_t off = 0, pending = nrows, id = row;
        for (uint32_t l = 0; l < nlevels; l++) {
            for (int k = 0; k < 4; k++) sibs[(q * nlevels + l) * 4 + k] = nodes[off + 4 * (id ^ 1) + k];
            off += 4 * pending;
            pending >>= 1;
            id >>= 1;
        }
    }
}

// ---------------------------------------------------------------- host side
static inline uint32_t blocks_for(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

// The permutation's tables are compile-time constants (poseidon_perm.hpp); nothing to upload.
int upload_poseidon_constants(Ctx &c)
{
    (void)c;
    return 0;
}

int poseidon_batch(uint64_t *out, const uint64_t *in, uint64_t n, int full, hipStream_t s)
{
    if (!n) return 0;
    hipLaunchKernelGGL(k_poseidon_batch, dim3(blocks_for(n, 256)), dim3(256), 0, s, out, in, n, full);
    return check_launch("k_poseidon_batch");
}

int merkle_leaves_cols(uint64_t *digests, const uint64_t *src, uint64_t ncols, uint64_t nrows, uint64_t ld,
                       hipStream_t s, const uint64_t *src2, uint64_t split)
{
    if (!nrows) return 0;
    prof_begin(s);
    if (src2 && split < ncols && ncols > 4)
        hipLaunchKernelGGL(k_leaves_cols2, dim3(blocks_for(nrows, 256)), dim3(256), 0, s, digests, src, ncols, nrows,
                           ld, src2, split);
    else
        hipLaunchKernelGGL(k_leaves_cols, dim3(blocks_for(nrows, 256)), dim3(256), 0, s, digests, src, ncols, nrows,
                           ld);
    prof_end("k_leaves_cols", 8.0 * (double)nrows * (double)ncols + 32.0 * (double)nrows, s);
    return check_launch("k_leaves_cols");
}

int merkle_leaves_rows(uint64_t *digests, const uint64_t *src, uint64_t ncols, uint64_t nrows, hipStream_t s)
{
    if (!nrows) return 0;
    prof_begin(s);
    if (nrows <= LP_MAX_PERMS && ncols > 4)
        hipLaunchKernelGGL(k_leaves_rows_lp, dim3(blocks_for(nrows * LP_LANES, 256)), dim3(256), 0, s, digests, src,
                           ncols, nrows);
    else
        hipLaunchKernelGGL(k_leaves_rows, dim3(blocks_for(nrows, 256)), dim3(256), 0, s, digests, src, ncols, nrows);
    prof_end("k_leaves_rows", 8.0 * (double)nrows * (double)ncols + 32.0 * (double)nrows, s);
    return check_launch("k_leaves_rows");
}

int merkle_levels(uint64_t *nodes, uint64_t nrows, hipStream_t s)
{
    uint64_t off = 0, pending = nrows;
    while (pending > 1) {
        uint64_t next = pending / 2;
        if (next <= LP_TAIL) {  // the remaining levels in one launch
            prof_begin(s);
            hipLaunchKernelGGL(k_merkle_tail_lp, dim3(1), dim3(1024), 0, s, nodes + off, pending);
            prof_end("k_merkle_level", 96.0 * (double)(pending - 1), s);
            break;
        }
        prof_begin(s);
        if (next <= LP_MAX_PERMS)
            hipLaunchKernelGGL(k_merkle_level_lp, dim3(blocks_for(next * LP_LANES, 256)), dim3(256), 0, s,
                               nodes + off + 4 * pending, nodes + off, next);
        else
            hipLaunchKernelGGL(k_merkle_level, dim3(blocks_for(next, 256)), dim3(256), 0, s, nodes + off + 4 * pending,
                               nodes + off, next);
        prof_end("k_merkle_level", 96.0 * (double)next, s);
        off += 4 * pending;
        pending = next;
    }
    return check_launch("k_merkle_level");
}

int merkle_open_strided(uint64_t *vals, uint64_t *sibs, const uint64_t *nodes, const uint64_t *src, uint64_t ncols,
                        uint64_t nrows, uint64_t row_stride, uint64_t col_stride, const uint64_t *idx, uint64_t nq,
                        hipStream_t s)
{
    if (!nq) return 0;
    uint32_t nlevels = 0;
    while ((1ULL << nlevels) < nrows) nlevels++;
    hipLaunchKernelGGL(k_merkle_open, dim3((uint32_t)nq), dim3(64), 0, s, vals, sibs, nodes, src, ncols, nrows,
                       row_stride, col_stride, idx, nq, nlevels);
    return check_launch("k_merkle_open");
}

int merkle_open_cols(uint64_t *vals, uint64_t *sibs, const uint64_t *nodes, const uint64_t *src, uint64_t ncols,
                     uint64_t nrows, uint64_t ld, const uint64_t *idx, uint64_t nq, hipStream_t s)
{
    return merkle_open_strided(vals, sibs, nodes, src, ncols, nrows, 1, ld, idx, nq, s);
}

}  // namespace zk
