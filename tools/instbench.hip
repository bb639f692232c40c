// Integer-instruction issue cost on gfx950 (wave64) at 1/2/4/8 waves per SIMD:
// the VALU peak that bench.py prices the field kernels against, and the
// basis for choosing the field arithmetic formulation.  8 independent chains per thread, inline asm pins
// the instruction.  Reports instructions/cycle/CU at the measured clock-free
// rate (ops per second / 256 CUs / 2.4e9).
// Build: hipcc -O3 --offload-arch=gfx950 -o build/instbench tools/instbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define ITERS 4096
#define STAMP() __builtin_amdgcn_s_memtime()

__global__ void k_mad_u64_u32(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3, b = blockIdx.x + 5;
    uint64_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++)
            asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b) : "s100", "s101");
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_mad_u32_u24(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3, b = blockIdx.x + 5;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_mul_lo_u32(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_mul_hi_u32(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_add64(uint64_t *out, int iters)
{
    uint64_t a = threadIdx.x + 3;
    uint64_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_add32(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_cmp64(uint64_t *out, int iters)
{
    uint64_t a = threadIdx.x + 3;
    uint64_t c[8];
    uint32_t acc = 0;
    for (int k = 0; k < 8; k++) c[k] = a * (k + 7);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            asm volatile("v_cmp_lt_u64 vcc, %0, %1" ::"v"(c[k]), "v"(a) : "vcc");
        }
    }
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((acc) & 1) << 63);
}

__global__ void k_bfi(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3, b = blockIdx.x;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(c[k]) : "v"(a), "v"(b));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}


__global__ void k_add_co(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_add_co_u32 %0, s[100:101], %0, %1" : "+v"(c[k]) : "v"(a) : "s100", "s101");
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

// v_addc_co_u32 reads a carry-in SGPR pair written once outside the loop
__global__ void k_addc_co(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    asm volatile("s_mov_b64 s[96:97], 0" ::: "s96", "s97");
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++)
            asm volatile("v_addc_co_u32 %0, s[100:101], %0, %1, s[96:97]" : "+v"(c[k]) : "v"(a) : "s100", "s101");
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_cndmask(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    asm volatile("s_mov_b64 s[96:97], 0x5555" ::: "s96", "s97");
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[96:97]" : "+v"(c[k]) : "v"(a));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_lshl64(uint64_t *out, int iters)
{
    uint64_t a = threadIdx.x + 3;
    uint64_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(c[k]));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_snop(uint64_t *out, int iters)
{
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("s_nop 0");
    }
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((iters) & 1) << 63);
}

__global__ void k_sub_co(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_sub_co_u32 %0, s[100:101], %0, %1" : "+v"(c[k]) : "v"(a) : "s100", "s101");
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_subbrev_co(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    asm volatile("s_mov_b64 s[96:97], 0" ::: "s96", "s97");
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++)
            asm volatile("v_subbrev_co_u32 %0, s[100:101], %0, %1, s[96:97]" : "+v"(c[k]) : "v"(a) : "s100", "s101");
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_mov(uint64_t *out, int iters)
{
    uint32_t a = threadIdx.x + 3;
    uint32_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 1);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_mov_b32 %0, %1" : "=v"(c[k]) : "v"(c[(k + 1) & 7]));
    }
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r ^= c[k];
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((r) & 1) << 63);
}

__global__ void k_cmp_gt64(uint64_t *out, int iters)
{
    uint64_t a = threadIdx.x + 3;
    uint64_t c[8];
    for (int k = 0; k < 8; k++) c[k] = a * (k + 7);
    const uint64_t t0_ = STAMP();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_cmp_gt_u64 vcc, %0, %1" ::"v"(c[k]), "v"(a) : "vcc");
    }
    const uint64_t t1_ = STAMP();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (t1_ - t0_) | ((uint64_t)((c[0]) & 1) << 63);
}

typedef void (*kfn)(uint64_t *, int);

int main()
{
    // Issue cost per wave64 instruction per SIMD at W waves per SIMD, clock-
    // free: every wave stamps s_memtime (shader cycles) around its loop of
    // ITERS x 8 independent instructions; with W waves sharing a SIMD the
    // SIMD issues W x ITERS x 8 instructions in a wave's lifetime T, so the
    // cost is T / (W x ITERS x 8) (median over waves).  256 threads per
    // workgroup (one wave per SIMD), 256*W workgroups (W per CU).
    const int maxw = 8;
    uint64_t *out;
    (void)hipMalloc(&out, 256ull * maxw * 256 * 8);
    std::vector<uint64_t> h(256ull * maxw * 256);
    struct {
        const char *name;
        kfn f;
    } ks[] = {{"v_add_u32", k_add32},        {"v_mad_u64_u32", k_mad_u64_u32}, {"v_add_co_u32", k_add_co},
              {"v_addc_co_u32", k_addc_co},   {"v_cndmask_b32", k_cndmask},     {"v_lshlrev_b64", k_lshl64},
              {"v_lshl_add_u64", k_add64},    {"v_mad_u32_u24", k_mad_u32_u24}, {"v_mul_lo_u32", k_mul_lo_u32},
              {"v_mul_hi_u32", k_mul_hi_u32}, {"v_cmp_lt_u64", k_cmp64},        {"v_bfi_b32", k_bfi},
              {"v_sub_co_u32", k_sub_co},     {"v_subbrev_co_u32", k_subbrev_co}, {"v_mov_b32", k_mov},
              {"v_cmp_gt_u64", k_cmp_gt64},   {"s_nop 0", k_snop}};
    const int waves[] = {1, 2, 4, 8};
    printf("{\"unit\": \"shader cycles per wave64 instruction per SIMD (s_memtime)\", \"rows\": [\n");
    bool first = true;
    for (int w : waves) {
        for (auto &k : ks) {
            const int blocks = 256 * w;
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, ITERS);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, ITERS);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h.data(), out, (size_t)blocks * 256 * 8, hipMemcpyDeviceToHost);
            std::vector<uint64_t> cyc;
            for (int b = 0; b < blocks; b++)
                for (int wv = 0; wv < 4; wv++) cyc.push_back(h[(size_t)b * 256 + wv * 64] & ~(1ULL << 63));
            std::sort(cyc.begin(), cyc.end());
            const double med = (double)cyc[cyc.size() / 2];
            const double cost = med / ((double)w * ITERS * 8);
            printf("%s  {\"instr\": \"%s\", \"waves_per_simd\": %d, \"cycles\": %.3f, \"wave_cycles_median\": %.0f}",
                   first ? "" : ",\n", k.name, w, cost, med);
            first = false;
        }
    }
    printf("\n]}\n");
    return 0;
}
