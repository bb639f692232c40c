// FETCH_SIZE calibration and re-read cost for the expression kernels' access
// shape (csrc/zxp_jit.hip: one row per lane, each column read as one u64 per
// lane from a column-major table, 512 contiguous bytes per wave load).
//
//   k_stream16<C>   16 B per lane, C columns read once (the shape the
//                   MI355X_MICROARCH.md correction is stated for)
//   k_cols8<C>      8 B per lane, C columns read once
//   k_reread<C, D>  8 B per lane, C columns in blocks of D, every block read
//                   twice back to back: each re-read comes D distinct columns
//                   after the first read of its column (the quotient's
//                   re-reads at stack distance D)
// Every kernel writes one u64 per row.  The launch holds 4 waves per SIMD (the
// segments' occupancy) through a 40 KB dynamic LDS allocation per workgroup.
// Printed: known bytes and GB/s per kernel; run it under
// `rocprofv3 --pmc FETCH_SIZE` (and WRITE_SIZE) to read the counters against
// the known byte counts.
// Build: hipcc -O3 --offload-arch=gfx950 -o build/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t ROWS = 1u << 24;
constexpr int NCOL = 128;
constexpr size_t LDS_PAD = 40 * 1024;

struct Cols {
    const uint64_t *c[NCOL];
};

template <int C>
__global__ __launch_bounds__(256) void k_cols8(Cols cols, uint64_t *out)
{
    extern __shared__ uint64_t pad[];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < C; j++) acc += cols.c[j][i];
    if (acc == 1) pad[threadIdx.x] = acc;  // keeps the LDS allocation
    out[i] = acc;
}

template <int C>
__global__ __launch_bounds__(256) void k_stream16(Cols cols, uint64_t *out)
{
    extern __shared__ uint64_t pad[];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;  // 2 rows per lane
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < C; j++) {
        const uint4 v = ((const uint4 *)cols.c[j])[i];
        acc += ((uint64_t)v.y << 32 | v.x) ^ ((uint64_t)v.w << 32 | v.z);
    }
    if (acc == 1) pad[threadIdx.x] = acc;
    out[i] = acc;
}

template <int C, int D>
__global__ __launch_bounds__(256) void k_reread(Cols cols, uint64_t *out)
{
    extern __shared__ uint64_t pad[];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint64_t acc = 0, acc2 = 0;
#pragma unroll
    for (int b = 0; b < C / D; b++) {
#pragma unroll
        for (int j = 0; j < D; j++) acc += cols.c[b * D + j][i];
        // a second load of the same cells (not a register copy), issued after
        // the block's first loads have landed (its address depends on them)
        const uint32_t i2 = i ^ (uint32_t)(acc == 0x123456789ULL);
#pragma unroll
        for (int j = 0; j < D; j++) acc2 ^= cols.c[b * D + j][i2];
    }
    if ((acc ^ acc2) == 1) pad[threadIdx.x] = acc;
    out[i] = acc ^ acc2;
}

template <typename K>
static double timed(K kern, uint32_t grid, Cols cols, uint64_t *out, double bytes, const char *name)
{
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), LDS_PAD, 0, cols, out);  // warm
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    for (int k = 0; k < 3; k++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), LDS_PAD, 0, cols, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= 3;
    printf("  \"%s\": {\"ms\": %.3f, \"bytes\": %.0f, \"GBps\": %.1f},\n", name, ms, bytes, bytes / (ms * 1e-3) / 1e9);
    return ms;
}

int main()
{
    uint64_t *buf, *out;
    if (hipMalloc(&buf, (size_t)NCOL * ROWS * 8) != hipSuccess || hipMalloc(&out, (size_t)ROWS * 8) != hipSuccess)
        return 1;
    (void)hipMemset(buf, 3, (size_t)NCOL * ROWS * 8);
    Cols cols;
    for (int j = 0; j < NCOL; j++) cols.c[j] = buf + (size_t)j * ROWS;
    const double col = (double)ROWS * 8, wr = (double)ROWS * 8;
    const uint32_t g = ROWS / 256;
    printf("{\n");
    timed(k_stream16<32>, g / 2, cols, out, 32 * col + wr / 2, "stream16_c32");
    timed(k_cols8<64>, g, cols, out, 64 * col + wr, "cols8_c64");
    timed(k_reread<64, 8>, g, cols, out, 128 * col + wr, "reread_d8");
    timed(k_reread<64, 16>, g, cols, out, 128 * col + wr, "reread_d16");
    timed(k_reread<64, 32>, g, cols, out, 128 * col + wr, "reread_d32");
    timed(k_reread<64, 64>, g, cols, out, 128 * col + wr, "reread_d64");
    timed(k_reread<128, 128>, g, cols, out, 256 * col + wr, "reread_d128");
    printf("  \"unique_read_bytes\": {\"stream16_c32\": %.0f, \"cols8_c64\": %.0f, \"reread\": %.0f, \"reread_d128\": %.0f}, \"write_bytes\": %.0f\n}\n",
           32 * col, 64 * col, 64 * col, 128 * col, wr);
    return 0;
}
