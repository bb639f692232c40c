// Integer-instruction throughput on gfx950 (wave64), for choosing the field
// arithmetic formulation.  8 independent chains per thread, inline asm pins
// the instruction.  Reports instructions/cycle/CU at the measured clock-free
// rate (ops per second / 256 CUs / 2.4e9).
// Build: hipcc -O3 --offload-arch=gfx950 -o build/instbench tools/instbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048

__global__ void k_mad_u64_u32(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3, b = blockIdx.x + 5;
    uint64_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++)
            asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b) : "s100", "s101");
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad_u32_u24(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3, b = blockIdx.x + 5;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_lo_u32(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_hi_u32(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_add64(uint64_t *out, int iters)
{
    uint64_t a = threadIdx.x + 3;
    uint64_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_add32(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_cmp64(uint64_t *out, int iters)
{
    uint64_t a = threadIdx.x + 3;
    uint64_t c[8];
    uint32_t acc = 0;
    for (int k = 0; k < 8; k++) c[k] = a * (k + 7);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            asm volatile("v_cmp_lt_u64 vcc, %0, %1" ::"v"(c[k]), "v"(a) : "vcc");
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_bfi(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3, b = blockIdx.x;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(c[k]) : "v"(a), "v"(b));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*kfn)(uint64_t *, int);

int main()
{
    uint64_t *out;
    (void)hipMalloc(&out, 2048 * 256 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct {
        const char *name;
        kfn f;
    } ks[] = {{"v_mad_u64_u32", k_mad_u64_u32}, {"v_mad_u32_u24", k_mad_u32_u24}, {"v_mul_lo_u32", k_mul_lo_u32},
              {"v_mul_hi_u32", k_mul_hi_u32},   {"v_lshl_add_u64", k_add64},     {"v_add_u32", k_add32},
              {"v_cmp_lt_u64", k_cmp64},        {"v_bfi_b32", k_bfi}};
    for (int rep = 0; rep < 2; rep++) {
        for (auto &k : ks) {
            hipLaunchKernelGGL(k.f, dim3(2048), dim3(256), 0, 0, out, ITERS);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(2048), dim3(256), 0, 0, out, ITERS);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            double ops = 2048.0 * 256 * ITERS * 8;  // lane-instructions
            double rate = ops / (ms * 1e-3);
            if (rep)
                printf("%-16s %8.2f T lane-op/s  = %.2f lane-op/clk/CU @2.4GHz (full rate = 128)\n", k.name,
                       rate / 1e12, rate / 256 / 2.4e9);
        }
    }
    return 0;
}
