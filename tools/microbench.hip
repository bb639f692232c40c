// Microbenchmarks on the MI355X: practical HBM copy bandwidth and the
// throughput of Goldilocks field-op variants (informs csrc/gl_device.hpp).
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o build/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../zkevm-prover_amd/csrc/gl_device.hpp"

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                       \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

using namespace zk;

__global__ void k_copy16(const uint4 *__restrict__ in, uint4 *__restrict__ out, size_t n)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) out[i] = in[i];
}

__global__ void k_copy8(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t n)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) out[i] = in[i];
}

// lazy variants ---------------------------------------------------------
__device__ __forceinline__ uint64_t red_lazy(uint64_t lo, uint64_t hi)
{
    uint32_t hh = (uint32_t)(hi >> 32), hl = (uint32_t)hi;
    uint64_t t0;
    bool b = __builtin_sub_overflow(lo, (uint64_t)hh, &t0);
    t0 -= b ? ZK_EPS : 0;
    uint64_t t1 = ((uint64_t)hl << 32) - hl;
    uint64_t r;
    bool c = __builtin_add_overflow(t0, t1, &r);
    r += c ? ZK_EPS : 0;
    return r;
}

__device__ __forceinline__ uint64_t mul_lazy(uint64_t a, uint64_t b)
{
    uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    uint64_t p00 = (uint64_t)a0 * b0;
    uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
    uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
    uint64_t hi = (uint64_t)a1 * b1 + (t >> 32) + (u >> 32);
    uint64_t lo = (u << 32) | (uint32_t)p00;
    return red_lazy(lo, hi);
}

template <int V>
__global__ void k_mul_chain(uint64_t *out, uint64_t seed, int iters)
{
    uint64_t x = seed + threadIdx.x + (uint64_t)blockIdx.x * 977;
    uint64_t y = x * 0x9E3779B97F4A7C15ULL;
    uint64_t z = y ^ 0x1234567ULL, w = z + 99;
    for (int i = 0; i < iters; i++) {
        if constexpr (V == 0) {
            x = gl_mul(x, y);
            z = gl_mul(z, w);
            y = gl_mul(y, x);
            w = gl_mul(w, z);
        } else {
            x = mul_lazy(x, y);
            z = mul_lazy(z, w);
            y = mul_lazy(y, x);
            w = mul_lazy(w, z);
        }
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = x ^ y ^ z ^ w;
}

template <int V>
__global__ void k_add_chain(uint64_t *out, uint64_t seed, int iters)
{
    uint64_t x = seed + threadIdx.x, y = x * 3 + 1, z = y * 5 + 7, w = z ^ 0xABCDEF;
    for (int i = 0; i < iters; i++) {
        x = gl_add(x, y);
        y = gl_sub(y, z);
        z = gl_add(z, w);
        w = gl_sub(w, x);
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = x ^ y ^ z ^ w;
}

int main()
{
    hipDevice_t dev;
    CHECK(hipGetDevice(&dev));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float ms;
    // ---- copy bandwidth, 4 GiB in / out
    size_t bytes = 4ULL << 30;
    void *a, *b;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMemset(a, 1, bytes));
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_copy16, dim3(256 * 8), dim3(256), 0, 0, (uint4 *)a, (uint4 *)b, bytes / 16);
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < 5; i++)
            hipLaunchKernelGGL(k_copy16, dim3(256 * 8), dim3(256), 0, 0, (uint4 *)a, (uint4 *)b, bytes / 16);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy16 : %.1f GB/s (read+write)\n", 2.0 * bytes * 5 / (ms * 1e-3) / 1e9);
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < 5; i++)
            hipLaunchKernelGGL(k_copy8, dim3(256 * 8), dim3(256), 0, 0, (uint64_t *)a, (uint64_t *)b, bytes / 8);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy8  : %.1f GB/s (read+write)\n", 2.0 * bytes * 5 / (ms * 1e-3) / 1e9);
    }
    // ---- field-op throughput
    uint64_t *out;
    CHECK(hipMalloc(&out, 256 * 1024 * 8 * sizeof(uint64_t)));
    const int iters = 4096;
    const int blocks = 256 * 8, threads = 256;
    double nthreads = (double)blocks * threads;
    for (int rep = 0; rep < 2; rep++) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_mul_chain<0>, dim3(blocks), dim3(threads), 0, 0, out, 7, iters);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("gl_mul (canonical): %.1f Gmul/s\n", nthreads * iters * 4 / (ms * 1e-3) / 1e9);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_mul_chain<1>, dim3(blocks), dim3(threads), 0, 0, out, 7, iters);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("mul_lazy          : %.1f Gmul/s\n", nthreads * iters * 4 / (ms * 1e-3) / 1e9);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_add_chain<0>, dim3(blocks), dim3(threads), 0, 0, out, 7, iters);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("gl_add/sub        : %.1f Gop/s\n", nthreads * iters * 4 / (ms * 1e-3) / 1e9);
    }
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(out));
    return 0;
}
