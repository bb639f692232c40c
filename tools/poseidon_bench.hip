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
    }
#pragma unroll
    for (int k = 0; k < 12; k++) st_all[k * n + i] = gl_canon(st[k]);
}

int main()
{
    const uint64_t n = 1 << 21;
    const int reps = 8;
    uint64_t *h = (uint64_t *)malloc(12 * n * 8), *ref = (uint64_t *)malloc(12 * n * 8), *o = (uint64_t *)malloc(12 * n * 8);
    uint64_t x = 0x5EED;
    for (uint64_t i = 0; i < 12 * n; i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        h[i] = x;  // includes non-canonical values
    }
    uint64_t *d;
    (void)hipMalloc(&d, 12 * n * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    typedef void (*kf)(uint64_t *, uint64_t, int);
    struct { const char *name; kf f; } ks[] = {
        {"textbook/halves (reference form)", k_perm<0>},
        {"textbook/limbs24", k_perm<1>},
        {"sparse/halves", k_perm<2>},
        {"sparse/limbs24", k_perm<3>},
        {"fast (folded MDS + block dots)", k_perm<4>},
    };
    int bad = 0;
    for (int v = 0; v < 5; v++) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            (void)hipMemcpy(d, h, 12 * n * 8, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(ks[v].f, dim3((uint32_t)(n / 256)), dim3(256), 0, 0, d, n, reps);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        (void)hipMemcpy(v ? o : ref, d, 12 * n * 8, hipMemcpyDeviceToHost);
        bool same = v == 0 || memcmp(o, ref, 12 * n * 8) == 0;
        bad |= !same;
        printf("%-34s %8.3f ms  %7.2f Gperm/s  %s\n", ks[v].name, best, (double)n * reps / (best * 1e-3) / 1e9,
               same ? "match" : "MISMATCH");
    }
    return bad;
}
