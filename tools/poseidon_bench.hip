// Poseidon-GL permutation variants on gfx950: throughput and cross-check.
// Each thread chains REPS permutations on its own state; all variants must
// produce the same final states as the textbook form with 32-bit-halves MDS
// (the reference's form).  Reports Gperm/s.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o build/poseidon_bench tools/poseidon_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../zkevm-prover_amd/csrc/poseidon_perm.hpp"

using namespace zk;

// previous MDS form (round 1 v3): plain C, the compiler strength-reduces the
// entries 2, 8, 16 into shift-adds and recombines with a 64-bit compare
__device__ __forceinline__ void mds_fold_v1(uint64_t st[12], const uint64_t *K)
{
    uint32_t lo[12], hi[12];
#pragma unroll
    for (int y = 0; y < 12; y++) {
        lo[y] = (uint32_t)st[y];
        hi[y] = (uint32_t)(st[y] >> 32);
    }
#pragma unroll
    for (int x = 0; x < 12; x++) {
        uint64_t sl = (uint32_t)K[x], sh = K[x] >> 32;
#pragma unroll
        for (int y = 0; y < 12; y++) {
            sl += (uint64_t)lo[y] * mds_entry(x, y);
            sh += (uint64_t)hi[y] * mds_entry(x, y);
        }
        uint64_t l;
        const bool c = __builtin_add_overflow(sl, sh << 32, &l);
        const uint32_t h = (uint32_t)(sh >> 32) + (c ? 1u : 0u);
        st[x] = gl_reduce96(l, h);
    }
}

__device__ __forceinline__ void full_rounds_fold_v1(uint64_t st[12], int r0)
{
#pragma unroll 1
    for (int r = r0; r < r0 + 4; r++) {
#pragma unroll
        for (int s = 0; s < 12; s++) st[s] = pow7(st[s]);
        const uint64_t *K = r == 3 ? ZKGPU_PSP_PRE : (r == 29 ? ZKGPU_PS_ZERO12 : &ZKGPU_POSEIDON_RC[(r + 1) * 12]);
        mds_fold_v1(st, K);
    }
}

// integer multiply-add MDS (mds_fold, 438 VALU) instead of the frequency-domain form
__device__ __forceinline__ void perm_fast_fold(uint64_t st[12])
{
#pragma unroll
    for (int s = 0; s < 12; s++) st[s] = gl_add(st[s], ZKGPU_POSEIDON_RC[s]);
    for (int h = 0; h < 2; h++) {
        if (h) partial_rounds_blocks(st);
        const int r0 = h ? 26 : 0;
#pragma unroll 1
        for (int r = r0; r < r0 + 4; r++) {
#pragma unroll
            for (int s = 0; s < 12; s++) st[s] = pow7(st[s]);
            const uint64_t *K = r == 3 ? ZKGPU_PSP_PRE : (r == 29 ? ZKGPU_PS_ZERO12 : &ZKGPU_POSEIDON_RC[(r + 1) * 12]);
            mds_fold(st, K);
        }
    }
}

__device__ __forceinline__ void perm_fast_v1(uint64_t st[12])
{
#pragma unroll
    for (int s = 0; s < 12; s++) st[s] = gl_add(st[s], ZKGPU_POSEIDON_RC[s]);
    full_rounds_fold_v1(st, 0);
    partial_rounds_blocks(st);
    full_rounds_fold_v1(st, 26);
}

template <int V>
__global__ void __launch_bounds__(256) k_perm(uint64_t *st_all, uint64_t n, int reps)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t st[12];
#pragma unroll
    for (int k = 0; k < 12; k++) st[k] = st_all[k * n + i];
    for (int r = 0; r < reps; r++) {
        if constexpr (V == 0) perm_textbook<false>(st);
        if constexpr (V == 1) perm_textbook<true>(st);
        if constexpr (V == 2) perm_sparse<false>(st);
        if constexpr (V == 3) perm_sparse<true>(st);
        if constexpr (V == 4) perm_fast(st);
        if constexpr (V == 5) perm_fast_fold(st);
        if constexpr (V == 6) perm_fast_v1(st);
        if constexpr (V == 7) {  // the 8 full rounds only (timing split)
            full_rounds_fold(st, 0);
            full_rounds_fold(st, 26);
        }
        if constexpr (V == 8) partial_rounds_blocks(st);  // the 22 partial rounds only
    }
#pragma unroll
    for (int k = 0; k < 12; k++) st_all[k * n + i] = gl_canon(st[k]);
}

// K states per thread (perm_fast_k): thread i owns states i + k * n / K
template <int K, bool SPLIT = false>
__global__ void __launch_bounds__(256) k_permK(uint64_t *st_all, uint64_t n, int reps)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t m = n / K;
    if (i >= m) return;
    uint64_t st[K][12];
#pragma unroll
    for (int k = 0; k < K; k++)
#pragma unroll
        for (int j = 0; j < 12; j++) st[k][j] = st_all[j * n + i + k * m];
    for (int r = 0; r < reps; r++) perm_fast_k<K, SPLIT>(st);
#pragma unroll
    for (int k = 0; k < K; k++)
#pragma unroll
        for (int j = 0; j < 12; j++) st_all[j * n + i + k * m] = gl_canon(st[k][j]);
}

// shader clock under the permutation load: s_memtime (shader cycles) against
// s_memrealtime (100 MHz) over each workgroup's lifetime
__global__ void __launch_bounds__(256) k_perm_clk(uint64_t *st_all, uint64_t n, int reps, uint64_t *clk)
{
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t st[12];
#pragma unroll
        for (int k = 0; k < 12; k++) st[k] = st_all[k * n + i];
        for (int r = 0; r < reps; r++) perm_fast(st);
#pragma unroll
        for (int k = 0; k < 12; k++) st_all[k * n + i] = gl_canon(st[k]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

// partial-round tables in memory: scalar loads (constant address space, not
// foldable) or staged into LDS per workgroup
__constant__ uint32_t g_psb_d0[759];
__constant__ uint32_t g_psb_bl[3828];

__global__ void __launch_bounds__(256) k_perm_smem(uint64_t *st_all, uint64_t n, int reps)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t st[12];
#pragma unroll
    for (int k = 0; k < 12; k++) st[k] = st_all[k * n + i];
    for (int r = 0; r < reps; r++) perm_fast_tab(st, g_psb_d0, g_psb_bl);
#pragma unroll
    for (int k = 0; k < 12; k++) st_all[k * n + i] = gl_canon(st[k]);
}

// the same with the table addresses opaque per permutation (no loop-invariant
// hoisting of the scalar loads out of the permutation loop)
typedef const __attribute__((address_space(4))) uint32_t c4u32;
__global__ void __launch_bounds__(256) k_perm_smem2(uint64_t *st_all, uint64_t n, int reps)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t st[12];
#pragma unroll
    for (int k = 0; k < 12; k++) st[k] = st_all[k * n + i];
    for (int r = 0; r < reps; r++) {
        c4u32 *d0 = (c4u32 *)g_psb_d0, *bl = (c4u32 *)g_psb_bl;
        asm volatile("" : "+s"(d0), "+s"(bl));
        perm_fast_tab(st, (const uint32_t *)d0, (const uint32_t *)bl);
    }
#pragma unroll
    for (int k = 0; k < 12; k++) st_all[k * n + i] = gl_canon(st[k]);
}

__global__ void __launch_bounds__(256) k_perm_lds(uint64_t *st_all, uint64_t n, int reps)
{
    __shared__ uint32_t d0[760], bl[3828];
    for (int k = threadIdx.x; k < 759; k += 256) d0[k] = g_psb_d0[k];
    for (int k = threadIdx.x; k < 3828; k += 256) bl[k] = g_psb_bl[k];
    __syncthreads();
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t st[12];
#pragma unroll
    for (int k = 0; k < 12; k++) st[k] = st_all[k * n + i];
    for (int r = 0; r < reps; r++) perm_fast_tab(st, d0, bl);
#pragma unroll
    for (int k = 0; k < 12; k++) st_all[k * n + i] = gl_canon(st[k]);
}

// occupancy targets: the product leaf kernel runs at 89 VGPRs = 5 waves/SIMD
template <int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, W))) k_perm_w(uint64_t *st_all, uint64_t n,
                                                                                             int reps)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t st[12];
#pragma unroll
    for (int k = 0; k < 12; k++) st[k] = st_all[k * n + i];
    for (int r = 0; r < reps; r++) perm_fast(st);
#pragma unroll
    for (int k = 0; k < 12; k++) st_all[k * n + i] = gl_canon(st[k]);
}

int main()
{
    const uint64_t n = 3 << 20;  // divisible by 2 and 3
    const int reps = 8;
    uint64_t *h = (uint64_t *)malloc(12 * n * 8), *ref = (uint64_t *)malloc(12 * n * 8), *o = (uint64_t *)malloc(12 * n * 8);
    uint64_t x = 0x5EED;
    for (uint64_t i = 0; i < 12 * n; i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        h[i] = x;  // includes non-canonical values
    }
    uint64_t *d;
    (void)hipMalloc(&d, 12 * n * 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_psb_d0), ZKGPU_PSB_D0, sizeof ZKGPU_PSB_D0);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_psb_bl), ZKGPU_PSB_BLOCKS, sizeof ZKGPU_PSB_BLOCKS);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    typedef void (*kf)(uint64_t *, uint64_t, int);
    struct { const char *name; kf f; } ks[] = {
        {"textbook/halves (reference form)", k_perm<0>},
        {"textbook/limbs24", k_perm<1>},
        {"sparse/halves", k_perm<2>},
        {"sparse/limbs24", k_perm<3>},
        {"fast (FFT MDS + block dots)", k_perm<4>},
        {"fast, multiply-add MDS (mds_fold)", k_perm<5>},
        {"fast, older MDS form", k_perm<6>},
        {"fast, K=1 generic (perm_fast_k)", k_permK<1>},
        {"fast, 2 states per thread", k_permK<2>},
        {"fast, split partial-round dots", k_permK<1, true>},
        {"fast, 2 states, split dots", k_permK<2, true>},
        {"fast, 6 waves/SIMD target", k_perm_w<6>},
        {"fast, 7 waves/SIMD target", k_perm_w<7>},
        {"fast, 8 waves/SIMD target", k_perm_w<8>},
        {"split: 8 full rounds only", k_perm<7>},
        {"split: 22 partial rounds only", k_perm<8>},
        {"fast, tables by scalar loads", k_perm_smem},
        {"fast, tables in LDS", k_perm_lds},
        {"fast, scalar loads, opaque table", k_perm_smem2},
    };
    const int nthreads_div[] = {1, 1, 1, 1, 1, 1, 1, 1, 2, 1, 2, 1, 1, 1, 1, 1, 1, 1, 1};
    int bad = 0;
    const int nv = sizeof(ks) / sizeof(ks[0]);
    for (int v = 0; v < nv; v++) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            (void)hipMemcpy(d, h, 12 * n * 8, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(ks[v].f, dim3((uint32_t)((n / nthreads_div[v] + 255) / 256)), dim3(256), 0, 0, d, n, reps);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        (void)hipMemcpy(v ? o : ref, d, 12 * n * 8, hipMemcpyDeviceToHost);
        bool same = v == 0 || v == 14 || v == 15 || memcmp(o, ref, 12 * n * 8) == 0;
        bad |= !same;
        printf("%-34s %8.3f ms  %7.2f Gperm/s  %s\n", ks[v].name, best, (double)n * reps / (best * 1e-3) / 1e9,
               same ? "match" : "MISMATCH");
    }
    {
        const uint32_t nb = (uint32_t)((n + 255) / 256);
        uint64_t *dclk, *hclk = (uint64_t *)malloc(2 * nb * 8);
        (void)hipMalloc(&dclk, 2 * nb * 8);
        (void)hipMemcpy(d, h, 12 * n * 8, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_perm_clk, dim3(nb), dim3(256), 0, 0, d, n, reps, dclk);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hclk, dclk, 2 * nb * 8, hipMemcpyDeviceToHost);
        double sc = 0, sr = 0;
        for (uint32_t b = 0; b < nb; b++) {
            sc += (double)hclk[2 * b];
            sr += (double)hclk[2 * b + 1];
        }
        printf("shader clock under load: %.3f GHz (s_memtime / s_memrealtime at 100 MHz, %u workgroups)\n",
               sc / (sr / 100e6) / 1e9, nb);
    }
    return bad;
}
