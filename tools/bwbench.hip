// HBM read efficiency by access granularity on gfx950, for the NTT pass
// design (tools/bwbench.hip): a four-step pass over a 2^k-point sub-DFT reads
// G consecutive u64 (one per "group") from each of many rows far apart, so
// each wave load instruction touches 64/G segments of 8*G bytes.  Measures
// GB/s of that gather (read) + a contiguous write, for G = 4, 8, 16, 32, and a
// plain streaming copy (the practical HBM peak the roofline quotes beside
// the 8 TB/s spec).
// Build: hipcc -O3 --offload-arch=gfx950 -o build/bwbench tools/bwbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// stream copy: 16 B per lane per access
__global__ void k_copy(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t n16)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

// segment gather: element (row r, group g) at in[r * stride + base + g];
// lanes: g = lane % G, r = lane / G (+ 64/G per iteration)
// NEAR: consecutive workgroups take neighbouring column blocks (they share
// 128 B lines and run at the same time); else neighbours are far apart in time
template <int G, bool NEAR>
__global__ void k_seg(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t rows, uint64_t stride)
{
    const uint64_t units = stride / G;  // column blocks of G
    const uint64_t rblocks = rows / ((256 / G) * 16);
    const uint64_t u = NEAR ? blockIdx.x % units : blockIdx.x / rblocks;
    const uint64_t rb = NEAR ? blockIdx.x / units : blockIdx.x % rblocks;  // row block of 256/G*16 rows
    const int g = threadIdx.x % G;
    const int r0 = threadIdx.x / G;
    constexpr int RPI = 256 / G;  // rows per iteration
    uint64_t acc = 0;
#pragma unroll 4
    for (int it = 0; it < 16; it++) {
        const uint64_t r = rb * (RPI * 16) + it * RPI + r0;
        if (r < rows) acc += in[r * stride + u * G + g];
    }
    out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int G, bool NEAR>
static double run_seg(const uint64_t *in, uint64_t *out, uint64_t rows, uint64_t stride)
{
    const uint64_t units = stride / G;
    const uint64_t rblocks = rows / ((256 / G) * 16);
    const dim3 grid((uint32_t)(units * rblocks));
    hipLaunchKernelGGL((k_seg<G, NEAR>), grid, dim3(256), 0, 0, in, out, rows, stride);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    for (int k = 0; k < 5; k++) hipLaunchKernelGGL((k_seg<G, NEAR>), grid, dim3(256), 0, 0, in, out, rows, stride);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double bytes = 5.0 * (rows * stride * 8.0 + units * rblocks * 256 * 8.0);
    return bytes / (ms * 1e-3) / 1e9;
}

int main()
{
    const uint64_t n = 1ULL << 30;  // 8 GiB of u64
    uint64_t *in, *out;
    if (hipMalloc(&in, n * 8) != hipSuccess || hipMalloc(&out, n * 8) != hipSuccess) return 1;
    (void)hipMemset(in, 1, n * 8);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const uint64_t n16 = n * 8 / 16 / 2;  // copy half the buffer into the other half
    hipLaunchKernelGGL(k_copy, dim3(256 * 64), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)out, n16);
    (void)hipEventRecord(a);
    for (int k = 0; k < 5; k++)
        hipLaunchKernelGGL(k_copy, dim3(256 * 64), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)out, n16);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("{\"copy_GBps\": %.1f", 5.0 * 2 * n16 * 16 / (ms * 1e-3) / 1e9);
    // rows x stride matrix of u64, stride 2^11 (16 KiB apart rows), 2^19 rows = 8 GiB
    const uint64_t stride = 1 << 11, rows = n / stride;
    printf(", \"seg_read_GBps_near\": {\"32B\": %.1f, \"64B\": %.1f, \"128B\": %.1f, \"256B\": %.1f}",
           run_seg<4, true>(in, out, rows, stride), run_seg<8, true>(in, out, rows, stride),
           run_seg<16, true>(in, out, rows, stride), run_seg<32, true>(in, out, rows, stride));
    printf(", \"seg_read_GBps_far\": {\"32B\": %.1f, \"64B\": %.1f, \"128B\": %.1f, \"256B\": %.1f}}\n",
           run_seg<4, false>(in, out, rows, stride), run_seg<8, false>(in, out, rows, stride),
           run_seg<16, false>(in, out, rows, stride), run_seg<32, false>(in, out, rows, stride));
    return 0;
}
