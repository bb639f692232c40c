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

// leaf digests from a column-major source (column c at src + c*ld)
__global__ void __launch_bounds__(256) k_leaves_cols(uint64_t *digests, const uint64_t *__restrict__ src,
                                                    uint64_t ncols, uint64_t nrows, uint64_t ld)
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
#pragma unroll
            for (int k = 0; k < 8; k++) st[k] = (uint64_t)k < nk ? src[(c0 + k) * ld + i] : 0;
            poseidon_perm(st);
        }
    }
    uint64_t *d = digests + 4 * i;
#pragma unroll
    for (int k = 0; k < 4; k++) d[k] = ncols <= 4 ? st[k] : gl_canon(st[k]);
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
                       hipStream_t s)
{
    if (!nrows) return 0;
    prof_begin(s);
    hipLaunchKernelGGL(k_leaves_cols, dim3(blocks_for(nrows, 256)), dim3(256), 0, s, digests, src, ncols, nrows, ld);
    prof_end("k_leaves_cols", 8.0 * (double)nrows * (double)ncols + 32.0 * (double)nrows, s);
    return check_launch("k_leaves_cols");
}

int merkle_leaves_rows(uint64_t *digests, const uint64_t *src, uint64_t ncols, uint64_t nrows, hipStream_t s)
{
    if (!nrows) return 0;
    prof_begin(s);
    hipLaunchKernelGGL(k_leaves_rows, dim3(blocks_for(nrows, 256)), dim3(256), 0, s, digests, src, ncols, nrows);
    prof_end("k_leaves_rows", 8.0 * (double)nrows * (double)ncols + 32.0 * (double)nrows, s);
    return check_launch("k_leaves_rows");
}

int merkle_levels(uint64_t *nodes, uint64_t nrows, hipStream_t s)
{
    uint64_t off = 0, pending = nrows;
    while (pending > 1) {
        uint64_t next = pending / 2;
        prof_begin(s);
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
