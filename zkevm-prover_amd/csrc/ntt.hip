// Goldilocks NTT / INTT / LDE kernels for gfx950 (column-major "SoA" layout).
//
// Replaces NTT_Goldilocks (submodule, absent) as used by the reference at
// starks.cpp:53,134,215 (extendPol), starks.cpp:262,285,326-327 (NTT/INTT).
// Semantics: natural order in and out, omega_n = W[log2 n], INTT scales 1/n,
// extendPol(out, in) = NTT_{n_ext}(zero_pad(INTT_n(in) * shift^i)).
//
// Algorithm (MI355X-first, see DESIGN.md "NTT"):
//   n = r_1 * r_2 * ... * r_P, each r_p = 2^b with 4 <= b <= 8 (n >= 2^13), a
//   Bailey/four-step recursion executed as P HBM passes.  Pass p takes
//   sub-DFTs of size r_p over stride m' = m / r_p inside blocks of size m,
//   multiplies by omega_m^{j' k} and writes back in place; the last pass
//   writes the digit-reversed result to its natural position.  Each
//   workgroup moves 16 independent sub-DFTs (16 consecutive j' = 128-byte
//   runs per row, so every global access is a full 128 B line), does the
//   radix-2 DIF butterflies in LDS and applies the twiddles on the way out.
//   Zero padding (LDE) is a predicated load in the first NTT pass; the
//   1/n * shift^k factor of the LDE is fused into the last INTT pass.
//   n <= 4096 uses a single-workgroup-per-column LDS kernel.
#include <stdlib.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "gl_device.hpp"
#include "gl_rb.hpp"
#include "zkgpu_internal.hpp"

namespace zk {

// ---------------------------------------------------------------- tables
// k_fill_powers: out[i] = scale * base^(i * step) for i < count
__global__ void k_fill_powers(uint64_t *out, uint64_t base, uint64_t step, uint64_t scale, uint64_t count)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint64_t b = gl_pow(base, step);
    out[i] = gl_canon(gl_mul(scale, gl_pow(b, i)));
}

__device__ __forceinline__ uint32_t bitrev_u32(uint32_t x, uint32_t bits)
{
    return bits == 0 ? 0 : (__builtin_bitreverse32(x) >> (32 - bits));
}

// omega_{2^TW_MAX_LOG}^e via the 2-level table (e < 2^TW_MAX_LOG)
__device__ __forceinline__ uint64_t tw_big(const uint64_t *lo, const uint64_t *hi, uint64_t e)
{
    return gl_mul(lo[e & (TW_LEVEL_SIZE - 1)], hi[e >> TW_LEVEL_BITS]);
}

// ---------------------------------------------------------------- pass kernel
struct PassArgs {
    const uint64_t *src;
    uint64_t src_ld;
    uint64_t src_valid;  // rows >= src_valid are zero (LDE padding)
    uint32_t half_zero;  // first pass of a zero-padded forward transform: inputs j1 >= R1/2 are zero
    uint64_t *dst;
    uint64_t dst_ld;
    const uint64_t *tw_lo;  // big twiddles omega_{2^28}, this direction
    const uint64_t *tw_hi;
    const uint64_t *post_lo;  // post-scale tables (last pass), may be null
    const uint64_t *post_hi;
    uint64_t post_step;   // post factor ratio between consecutive k2 (last pass)
    uint64_t post_scale;  // applied when post_lo == null and != 1
    uint32_t post_bits;
    uint32_t logn;
    uint32_t logm;  // block size before this pass (first pass: logn)
    uint32_t last;  // 1 = last pass (digit-reversed scatter)
    uint32_t npass;
    uint32_t rbits[NTT_MAX_PASSES];
    const uint64_t *otw;  // outer twiddles omega_m^(j' k) at [k << logmp | j'] (null: recurrence)
    const uint64_t *rt4096;  // omega_4096^e, e < 4096, this direction (the pass's omega_R table)
    uint32_t ncols;       // columns in this launch (grid x = unit * ncols + column)
};

constexpr int GROUPS = 16;

// radix-2 DIF network on R = 2^LOG registers; afterwards v[r] = X[bitrev(r)].
// twiddle omega_{2h}^i = 2^e with e = 96 i / h in [0, 96) (forward); the
// inverse twiddle 2^(192 - e) = -2^(96 - e), so the inverse butterfly
// computes (c - a) * 2^(96 - e) and never needs a negation.
// RB: the butterflies' add / sub with the rare second carry behind a
// wave-uniform branch (gl_add_rb / gl_sub_rb, csrc/gl_device.hpp): 5 + 7
// VALU instead of 7 + 10.  The radix-256 pass kernel uses it (LDE 52.8 ->
// 56.9 Gelem/s); the 3-pass LDE's 64-register kernels do not (their branchy
// form ran at half speed: 49.1 -> 26.0 Gelem/s).  ZKGPU_NTT_RB=0 builds the
// select form everywhere.
#ifndef ZKGPU_NTT_RB
#define ZKGPU_NTT_RB 1
#endif
#ifndef ZKGPU_NTT_RB_SHIFT  // the shift-multiplies' rare corrections too (mul2e_rb)
#define ZKGPU_NTT_RB_SHIFT 1
#endif
template <bool RB>
__device__ __forceinline__ uint64_t bf_add(uint64_t a, uint64_t b)
{
    if constexpr (RB && ZKGPU_NTT_RB) return gl_add_rb(a, b);
    else return gl_add(a, b);
}
template <bool RB>
__device__ __forceinline__ uint64_t bf_sub(uint64_t a, uint64_t b)
{
    if constexpr (RB && ZKGPU_NTT_RB) return gl_sub_rb(a, b);
    else return gl_sub(a, b);
}

template <int E, bool RB>
__device__ __forceinline__ uint64_t bf_mul2e(uint64_t x)
{
    if constexpr (RB && ZKGPU_NTT_RB && ZKGPU_NTT_RB_SHIFT) return mul2e_rb<E>(x);
    else return mul2e<E>(x);
}

template <bool INV, int H, int I, bool RB>
__device__ __forceinline__ uint64_t dif_odd(uint64_t a, uint64_t c)
{
    constexpr int e = (96 * I) / H;
    if constexpr (e == 0) return bf_sub<RB>(a, c);
    else if constexpr (!INV) return bf_mul2e<e, RB>(bf_sub<RB>(a, c));
    else return bf_mul2e<96 - e, RB>(bf_sub<RB>(c, a));
}

template <int LOG, bool INV, bool RB = false, int H = (1 << LOG) / 2>
__device__ __forceinline__ void dft_regs(uint64_t *v)
{
    if constexpr (H >= 1) {
        constexpr int R = 1 << LOG;
        [&]<int... Bs>(std::integer_sequence<int, Bs...>) {
            (
                [&]<int B>() {
                    [&]<int... Is>(std::integer_sequence<int, Is...>) {
                        (
                            [&]<int I>() {
                                uint64_t a = v[B * 2 * H + I];
                                uint64_t c = v[B * 2 * H + I + H];
                                v[B * 2 * H + I] = bf_add<RB>(a, c);
                                v[B * 2 * H + I + H] = dif_odd<INV, H, I, RB>(a, c);
                            }.template operator()<Is>(),
                            ...);
                    }(std::make_integer_sequence<int, H>{});
                }.template operator()<Bs>(),
                ...);
        }(std::make_integer_sequence<int, R / (2 * H)>{});
        dft_regs<LOG, INV, RB, H / 2>(v);
    }
}

// dft_regs when the upper half of v[] is zero (the zero-padded LDE input):
// the first stage's butterflies are (a, 0) -> (a, a * 2^e), exactly what
// gl_add(a, 0) / gl_sub(a, 0) return, without the adds
template <int LOG, bool INV, bool RB = false>
__device__ __forceinline__ void dft_regs_half(uint64_t *v)
{
    constexpr int R = 1 << LOG, H = R / 2;
    [&]<int... Is>(std::integer_sequence<int, Is...>) {
        ([&]<int I>() {
            constexpr int e = (96 * I) / H;
            static_assert(!INV, "forward only");
            if constexpr (e == 0) v[I + H] = v[I];
            else v[I + H] = mul2e<e>(v[I]);
        }.template operator()<Is>(), ...);
    }(std::make_integer_sequence<int, H>{});
    dft_regs<LOG, INV, RB, H / 2>(v);
}

__host__ __device__ constexpr int brev_c(int x, int bits)
{
    int r = 0;
    for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
    return r;
}

// One pass of radix R = 2^(L1+L2) over 16 independent sub-DFTs per workgroup.
//   step 1: thread (g, j2) loads x[R2*j1 + j2] (j1 < R1), R1-point DFT in
//           registers, times omega_R^(j2*k1), to LDS
//   step 2: thread (g, k1) reads y[j2][k1] (j2 < R2), R2-point DFT in
//           registers -> X[k1 + R1*k2], outer twiddle / post-scale, store.
// LDS image (k1*R2 + j2)*17 + g: conflict-free for both access patterns.
// SPLIT: the LDS transpose moves the low and then the high 32-bit words
// through a half-size image (two more barriers), halving the workgroup's LDS
// so more waves fit per CU (LDS, not VGPRs, limits the radix-256 pass).
template <int L1, int L2, bool INV, bool SPLIT>
__global__ void __launch_bounds__(16 * (1 << L2)) k_ntt_pass(PassArgs a)
{
    constexpr int R1 = 1 << L1, R2 = 1 << L2, LOGR = L1 + L2, R = 1 << LOGR;
    constexpr int T = GROUPS * R2;
    __shared__ uint64_t lds[SPLIT ? R * 8 : R * 17];
    uint32_t *lds32 = reinterpret_cast<uint32_t *>(lds);
    // SPLIT image: row rho = k1 * R2 + j2 holds the 16 groups' words; row
    // rho is stored at rho ^ (bit L2 of rho), so both 32-lane groups of
    // ds_write_b32 (two consecutive j2) and of ds_read_b32 (two consecutive
    // k1) cover the 32 banks once: conflict-free, no padding

    __shared__ uint64_t twR[R];  // omega_R^i
    // columns vary fastest across workgroups: the workgroups sharing a unit's
    // outer-twiddle slice run together and find it in L2
    const uint32_t col = blockIdx.x % a.ncols;
    const uint64_t u = blockIdx.x / a.ncols;
    const uint64_t *src = a.src + (uint64_t)col * a.src_ld;
    uint64_t *dst = a.dst + (uint64_t)col * a.dst_ld;
    const int tid = threadIdx.x;

    // omega_R^i = omega_4096^(i << (12 - LOGR)) (R <= 256)
    static_assert(LOGR <= 12, "radix");
    if (a.rt4096)
        for (int i = tid; i < R; i += T) twR[i] = a.rt4096[i << (12 - LOGR)];
    else
        for (int i = tid; i < R; i += T) twR[i] = tw_big(a.tw_lo, a.tw_hi, (uint64_t)i << (TW_MAX_LOG - LOGR));

    uint64_t v[R2 > R1 ? R2 : R1];
    // ------------------------------------------------ step 1 (load + R1-DFT)
    int g, j2;
    uint64_t base = 0, k1g = 0, rest = 0;
    uint32_t logmp = 0, logS = 0;
    if (!a.last) {
        g = tid & 15;
        j2 = tid >> 4;
        logmp = a.logm - LOGR;
        const uint64_t groups_per_blk = 1ULL << (logmp - 4);
        const uint64_t blk = u >> (logmp - 4);
        const uint64_t j0 = (u & (groups_per_blk - 1)) << 4;
        base = (blk << a.logm) + j0;
#pragma unroll
        for (int j1 = 0; j1 < R1; j1++) {
            uint64_t pos = base + ((uint64_t)(R2 * j1 + j2) << logmp) + g;
            v[j1] = pos < a.src_valid ? src[pos] : 0;
        }
    } else {
        j2 = tid & (R2 - 1);
        g = tid >> L2;
        logS = a.logn - a.rbits[0] - LOGR;
        rest = u & ((1ULL << logS) - 1);
        k1g = u >> logS;
        const uint64_t blk = ((k1g * 16 + g) << logS) + rest;
#pragma unroll
        for (int j1 = 0; j1 < R1; j1++) {
            uint64_t pos = (blk << LOGR) + R2 * j1 + j2;
            v[j1] = pos < a.src_valid ? src[pos] : 0;
        }
    }
    if constexpr (!INV) {
        if (a.half_zero)
            dft_regs_half<L1, INV, true>(v);
        else
            dft_regs<L1, INV, true>(v);
    } else {
        dft_regs<L1, INV, true>(v);
    }
    __syncthreads();  // twR ready
#pragma unroll
    for (int r = 0; r < R1; r++) {
        const int k1 = brev_c(r, L1);
        if (k1) v[r] = gl_mul_rb(v[r], twR[(j2 * k1) & (R - 1)]);
    }
    const bool active = tid < GROUPS * R1;  // step-2 threads
    const int g2 = tid & 15, k1s = tid >> 4;
    if constexpr (SPLIT) {
        uint32_t lo[R2 > R1 ? R2 : R1];
        // write: row brev(r) * R2 + j2 -> flip = bit 0 of brev(r) (R2 even): two bases
        const int wb0 = (j2 << 4) + g, wb1 = ((j2 ^ 1) << 4) + g;
        // read: row k1s * R2 + jj -> flip = k1s & 1: slot = k1s*R2*16 + ((jj ^ f) << 4) + g2
        const int fm = (k1s & 1) << 4;
        const int rbe = k1s * R2 * 16 + g2 + fm, rbo = k1s * R2 * 16 + g2 - fm;
#pragma unroll
        for (int r = 0; r < R1; r++) {
            const int k1 = brev_c(r, L1);
            lds32[k1 * R2 * 16 + ((k1 & 1) ? wb1 : wb0)] = (uint32_t)v[r];
        }
        __syncthreads();
        if (active) {
#pragma unroll
            for (int jj = 0; jj < R2; jj++) lo[jj] = lds32[((jj & 1) ? rbo : rbe) + (jj << 4)];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R1; r++) {
            const int k1 = brev_c(r, L1);
            lds32[k1 * R2 * 16 + ((k1 & 1) ? wb1 : wb0)] = (uint32_t)(v[r] >> 32);
        }
        __syncthreads();
        if (!active) return;
#pragma unroll
        for (int jj = 0; jj < R2; jj++) v[jj] = ((uint64_t)lds32[((jj & 1) ? rbo : rbe) + (jj << 4)] << 32) | lo[jj];
    } else {
#pragma unroll
        for (int r = 0; r < R1; r++) lds[(brev_c(r, L1) * R2 + j2) * 17 + g] = v[r];
        __syncthreads();
        if (!active) return;
#pragma unroll
        for (int jj = 0; jj < R2; jj++) v[jj] = lds[(k1s * R2 + jj) * 17 + g2];
    }
    // ------------------------------------------------ step 2 (R2-DFT + store)
    g = g2;
    const int k1 = k1s;
    dft_regs<L2, INV, true>(v);
    if (!a.last && a.otw) {
        // X[k] * omega_m^(j' k) from the table (one coalesced load per element
        // instead of a recurrence product), k = k1 + R1*k2, j' = j0 + g
        const uint64_t jp = (base & ((1ULL << logmp) - 1)) + g;
#pragma unroll
        for (int k2 = 0; k2 < R2; k2++) {
            const int r = brev_c(k2, L2);
            const uint64_t k = (uint64_t)(k1 + R1 * k2);
            uint64_t x = v[r];
            if (k1 | k2) x = gl_mul_rb(x, a.otw[(k << logmp) + jp]);
            dst[base + (k << logmp) + g] = x;  // intermediate: lazy
        }
    } else if (!a.last) {
        // X[k] * omega_m^(j' k), k = k1 + R1*k2, j' = j0 + g
        const uint32_t tshift = TW_MAX_LOG - a.logm;
        const uint64_t jp = (base & ((1ULL << logmp) - 1)) + g;
        uint64_t t = tw_big(a.tw_lo, a.tw_hi, (jp * k1) << tshift);
        const uint64_t step = tw_big(a.tw_lo, a.tw_hi, (jp * R1) << tshift);
#pragma unroll
        for (int k2 = 0; k2 < R2; k2++) {
            const int r = brev_c(k2, L2);
            uint64_t x = v[r];
            if (k1 | k2) x = gl_mul(x, t);
            dst[base + ((uint64_t)(k1 + R1 * k2) << logmp) + g] = x;  // intermediate: lazy
            t = gl_mul(t, step);
        }
    } else {
        uint64_t rrev = 0;
        {
            // rest = sum_{i=1..npass-2} k_i * prod_{l>i} r_l; rrev = mixed-radix reversal
            uint32_t rev_pos[NTT_MAX_PASSES];
            uint32_t acc = 0;
            for (uint32_t i = 1; i + 1 < a.npass; i++) {
                rev_pos[i] = acc;
                acc += a.rbits[i];
            }
            uint64_t rr = rest;
            for (int i = (int)a.npass - 2; i >= 1; i--) {
                uint64_t d = rr & ((1ULL << a.rbits[i]) - 1);
                rr >>= a.rbits[i];
                rrev |= d << rev_pos[i];
            }
        }
        const uint32_t lognr = a.logn - LOGR;
        const uint64_t x0 = (k1g * 16 + g) + (rrev << a.rbits[0]) + ((uint64_t)k1 << lognr);
        const bool scaled = a.post_lo != nullptr || a.post_scale != 1;
        uint64_t f = a.post_scale;
        if (a.post_lo) f = gl_mul(a.post_lo[x0 & ((1ULL << a.post_bits) - 1)], a.post_hi[x0 >> a.post_bits]);
#pragma unroll
        for (int k2 = 0; k2 < R2; k2++) {
            const int r = brev_c(k2, L2);
            uint64_t x = v[r];
            if (scaled) x = gl_mul(x, f);
            dst[x0 + ((uint64_t)(R1 * k2) << lognr)] = gl_canon(x);
            if (a.post_lo) f = gl_mul(f, a.post_step);
        }
    }
}

// ---------------------------------------------------------------- small NTT
// one workgroup per column, whole column (n <= 4096) in LDS
constexpr int PASS_THREADS = 256;

struct SmallArgs {
    const uint64_t *src;
    uint64_t src_ld;
    uint64_t src_valid;
    uint64_t *dst;
    uint64_t dst_ld;
    const uint64_t *rt_small;
    const uint64_t *post_lo;
    const uint64_t *post_hi;
    uint64_t post_scale;
    uint32_t post_bits;
    uint32_t logn;
};

__global__ void __launch_bounds__(PASS_THREADS) k_ntt_small(SmallArgs a)
{
    __shared__ uint64_t lds[4096];
    const uint32_t col = blockIdx.x;
    const uint64_t *src = a.src + (uint64_t)col * a.src_ld;
    uint64_t *dst = a.dst + (uint64_t)col * a.dst_ld;
    const uint32_t n = 1u << a.logn;
    for (uint32_t i = threadIdx.x; i < n; i += PASS_THREADS) lds[i] = i < a.src_valid ? src[i] : 0;
    for (int lh = (int)a.logn - 1; lh >= 0; lh--) {
        const uint32_t h = 1u << lh;
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < n / 2; b += PASS_THREADS) {
            uint32_t pos = b & (h - 1);
            uint32_t i0 = ((b >> lh) << (lh + 1)) + pos;
            uint32_t i1 = i0 + h;
            uint64_t x = lds[i0], y = lds[i1];
            lds[i0] = gl_add(x, y);
            uint64_t d = gl_sub(x, y);
            // omega_{2h}^pos = omega_4096^(pos * 4096/(2h))
            lds[i1] = pos == 0 ? d : gl_mul(d, a.rt_small[pos << (11 - lh)]);
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < n; k += PASS_THREADS) {
        uint64_t v = lds[bitrev_u32(k, a.logn)];
        if (a.post_lo)
            v = gl_mul(v, gl_mul(a.post_lo[k & ((1u << a.post_bits) - 1)], a.post_hi[k >> a.post_bits]));
        else if (a.post_scale != 1)
            v = gl_mul(v, a.post_scale);
        dst[k] = gl_canon(v);
    }
}

// ---------------------------------------------------------------- transpose
// row-major (nrows x ncols, row stride ncols) <-> column-major (ld per column)
__global__ void k_rows_to_cols(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t nrows,
                               uint64_t ncols, uint64_t ld)
{
    __shared__ uint64_t tile[32][33];
    uint64_t r0 = (uint64_t)blockIdx.x * 32, c0 = (uint64_t)blockIdx.y * 32;
    int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
    for (int k = ty; k < 32; k += 8) {
        uint64_t r = r0 + k, c = c0 + tx;
        if (r < nrows && c < ncols) tile[k][tx] = in[r * ncols + c];
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        uint64_t c = c0 + k, r = r0 + tx;
        if (r < nrows && c < ncols) out[c * ld + r] = tile[tx][k];
    }
}

__global__ void k_cols_to_rows(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t nrows,
                               uint64_t ncols, uint64_t ld)
{
    __shared__ uint64_t tile[32][33];
    uint64_t r0 = (uint64_t)blockIdx.x * 32, c0 = (uint64_t)blockIdx.y * 32;
    int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int k = ty; k < 32; k += 8) {
        uint64_t c = c0 + k, r = r0 + tx;
        if (r < nrows && c < ncols) tile[k][tx] = in[c * ld + r];
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        uint64_t r = r0 + k, c = c0 + tx;
        if (r < nrows && c < ncols) out[r * ncols + c] = tile[tx][k];
    }
}

// outer twiddle table of a pass over blocks of m = 2^logm with sub-DFT size
// R = 2^logr: out[k << (logm - logr) | j'] = omega_m^(j' k), k < R, j' < m / R
__global__ void k_otw_table(uint64_t *out, const uint64_t *tw_lo, const uint64_t *tw_hi, uint32_t logm,
                            uint32_t logr)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >> logm) return;
    const uint32_t logmp = logm - logr;
    const uint64_t k = i >> logmp, jp = i & ((1ULL << logmp) - 1);
    out[i] = gl_canon(tw_big(tw_lo, tw_hi, (jp * k) << (TW_MAX_LOG - logm)));
}

// ---------------------------------------------------------------- host side
// Outer-twiddle tables, built on first use per (direction, log m, log R) and
// kept for the process (<= 2^OTW_MAX_LOG entries each; 128 MB at 2^24).
constexpr uint32_t OTW_MAX_LOG = 24;
struct OtwTable {
    int d;
    uint32_t logm, logr;
    uint64_t *ptr;
};
static std::vector<OtwTable> g_otw;

static const uint64_t *otw_table(Ctx &ctx, int d, uint32_t logm, uint32_t logr, hipStream_t s)
{
    if (logm > OTW_MAX_LOG) return nullptr;
    for (const OtwTable &t : g_otw)
        if (t.d == d && t.logm == logm && t.logr == logr) return t.ptr;
    uint64_t *p = nullptr;
    const uint64_t m = 1ULL << logm;
    if (hipMalloc((void **)&p, m * sizeof(uint64_t)) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;  // no memory for the table: the recurrence path is exact too
    }
    hipLaunchKernelGGL(k_otw_table, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, s, p, ctx.tw_lo[d], ctx.tw_hi[d],
                       logm, logr);
    g_otw.push_back(OtwTable{d, logm, logr, p});
    return p;
}

// live-profiling labels: radix and direction (the forward and inverse
// instantiations are different kernels with different traffic)
static const char *PASS_NAMES[2][9] = {
    {"", "", "", "", "k_ntt_pass<4,fwd>", "k_ntt_pass<5,fwd>", "k_ntt_pass<6,fwd>", "k_ntt_pass<7,fwd>",
     "k_ntt_pass<8,fwd>"},
    {"", "", "", "", "k_ntt_pass<4,inv>", "k_ntt_pass<5,inv>", "k_ntt_pass<6,inv>", "k_ntt_pass<7,inv>",
     "k_ntt_pass<8,inv>"}};

static void split_radix(uint32_t logn, uint32_t *npass, uint32_t rbits[NTT_MAX_PASSES])
{
    uint32_t P = (logn + 7) / 8;
    *npass = P;
    uint32_t base = logn / P, extra = logn % P;
    // larger radices last (the last pass reads contiguous runs of R)
    for (uint32_t i = 0; i < P; i++) rbits[i] = base + (i >= P - extra ? 1 : 0);
}

template <int L1, int L2>
static void launch_pass(const PassArgs &a, uint64_t ncols, int inverse, hipStream_t s)
{
    constexpr int LOGR = L1 + L2;
    uint64_t units = (1ULL << (a.logn - LOGR)) / 16;
    dim3 grid((uint32_t)(units * ncols));
    if (inverse)
        hipLaunchKernelGGL((k_ntt_pass<L1, L2, true, true>), grid, dim3(16 << L2), 0, s, a);
    else
        hipLaunchKernelGGL((k_ntt_pass<L1, L2, false, true>), grid, dim3(16 << L2), 0, s, a);
}

static void dispatch_pass(uint32_t logr, const PassArgs &a, uint64_t ncols, int inverse, hipStream_t s)
{
    switch (logr) {
    case 4: launch_pass<2, 2>(a, ncols, inverse, s); break;
    case 5: launch_pass<2, 3>(a, ncols, inverse, s); break;
    case 6: launch_pass<3, 3>(a, ncols, inverse, s); break;
    case 7: launch_pass<3, 4>(a, ncols, inverse, s); break;
    case 8: launch_pass<4, 4>(a, ncols, inverse, s); break;
    default: break;
    }
}

// One full transform over ncols columns.
//   src: column c at src + c*src_ld, src_valid rows (rest zero)
//   dst: column c at dst + c*dst_ld, n rows, natural order
//   tmp: scratch, column c at tmp + c*tmp_ld (tmp_ld >= n), only for n > 4096
//   post: optional per-row factor tables (last pass)
int ntt_columns(Ctx &ctx, uint64_t *dst, uint64_t dst_ld, const uint64_t *src, uint64_t src_ld, uint64_t src_valid,
                uint64_t *tmp, uint64_t tmp_ld, uint32_t logn, uint64_t ncols, int inverse, const uint64_t *post_lo,
                const uint64_t *post_hi, uint32_t post_bits, uint64_t post_base, uint64_t post_scale, hipStream_t s)
{
    if (ncols == 0) return 0;
    if (logn > TW_MAX_LOG) return set_error(ZKGPU_ERR_ARG, "ntt: log2(n) exceeds %u", TW_MAX_LOG);
    const int d = inverse ? 1 : 0;
    if (logn <= 12) {
        SmallArgs sa;
        sa.src = src;
        sa.src_ld = src_ld;
        sa.src_valid = src_valid;
        sa.dst = dst;
        sa.dst_ld = dst_ld;
        sa.rt_small = ctx.rt_small[d];
        sa.post_lo = post_lo;
        sa.post_hi = post_hi;
        sa.post_bits = post_bits;
        sa.post_scale = post_scale;
        sa.logn = logn;
        for (uint64_t c0 = 0; c0 < ncols; c0 += 65535) {
            uint64_t nc = ncols - c0 < 65535 ? ncols - c0 : 65535;
            SmallArgs b = sa;
            b.src = src + c0 * src_ld;
            b.dst = dst + c0 * dst_ld;
            const uint64_t n = 1ULL << logn;
            const uint64_t nread = (src_valid < n ? src_valid : n);
            prof_begin(s);
            hipLaunchKernelGGL(k_ntt_small, dim3((uint32_t)nc), dim3(PASS_THREADS), 0, s, b);
            prof_end("k_ntt_small", 8.0 * (double)(nread + n) * (double)nc, s);
        }
        return check_launch("k_ntt_small");
    }
    PassArgs a;
    a.rt4096 = ctx.rt_small[d];  // omega_R from the table (+0.6 % against the 2-level product)
    a.tw_lo = ctx.tw_lo[d];
    a.tw_hi = ctx.tw_hi[d];
    a.logn = logn;
    split_radix(logn, &a.npass, a.rbits);
    uint32_t logm = logn;
    for (uint32_t p = 0; p < a.npass; p++) {
        a.logm = logm;
        a.last = (p == a.npass - 1);
        a.post_lo = a.last ? post_lo : nullptr;
        a.post_hi = a.last ? post_hi : nullptr;
        a.post_bits = post_bits;
        a.post_scale = a.last ? post_scale : 1;
        // factor ratio between outputs k1 + R1*k2 and k1 + R1*(k2+1): base^(R1 * n/R)
        const uint32_t rb = a.rbits[p];
        a.post_step = h_pow(post_base, (uint64_t)(1u << (rb / 2)) << (logn - rb));
        a.otw = a.last ? nullptr : otw_table(ctx, d, logm, rb, s);
        a.half_zero = 0;
        if (p == 0) {
            a.src = src;
            a.src_ld = src_ld;
            a.src_valid = src_valid;
            // zero-padded forward input: exactly the rows j1 >= R1/2 of every
            // sub-DFT (positions (R2 j1 + j2) * n / R) are past src_valid
            const uint32_t l1 = rb / 2;  // launch_pass<L1 = rb/2, L2 = rb - L1>
            a.half_zero = (!inverse && l1 >= 1 && src_valid == (1ULL << (logn - 1))) ? 1u : 0u;
        } else {
            a.src = tmp;
            a.src_ld = tmp_ld;
            a.src_valid = ~0ULL;
        }
        if (a.last) {
            a.dst = dst;
            a.dst_ld = dst_ld;
        } else {
            a.dst = tmp;
            a.dst_ld = tmp_ld;
        }
        const uint64_t n = 1ULL << logn;
        const uint64_t nread = (a.src_valid < n ? a.src_valid : n);
        // columns per launch: grid x = units * columns, at most 2^32 threads
        const uint64_t units = (1ULL << (logn - rb)) / 16;
        const uint64_t cmax = std::max<uint64_t>(1, std::min<uint64_t>(65535, (1ULL << 32) / (units * 256)));
        for (uint64_t c0 = 0; c0 < ncols; c0 += cmax) {
            uint64_t nc = ncols - c0 < cmax ? ncols - c0 : cmax;
            PassArgs b = a;
            b.src = a.src + c0 * a.src_ld;
            b.dst = a.dst + c0 * a.dst_ld;
            b.ncols = (uint32_t)nc;
            prof_begin(s);
            dispatch_pass(rb, b, nc, inverse, s);
            prof_end(PASS_NAMES[d][rb], 8.0 * (double)(nread + n) * (double)nc, s);
        }
        logm -= rb;
    }
    return check_launch("k_ntt_pass");
}

void rows_to_cols(const uint64_t *in, uint64_t *out, uint64_t nrows, uint64_t ncols, uint64_t ld, hipStream_t s)
{
    if (!nrows || !ncols) return;
    dim3 grid((uint32_t)((nrows + 31) / 32), (uint32_t)((ncols + 31) / 32));
    hipLaunchKernelGGL(k_rows_to_cols, grid, dim3(256), 0, s, in, out, nrows, ncols, ld);
}

void cols_to_rows(const uint64_t *in, uint64_t *out, uint64_t nrows, uint64_t ncols, uint64_t ld, hipStream_t s)
{
    if (!nrows || !ncols) return;
    dim3 grid((uint32_t)((nrows + 31) / 32), (uint32_t)((ncols + 31) / 32));
    hipLaunchKernelGGL(k_cols_to_rows, grid, dim3(256), 0, s, in, out, nrows, ncols, ld);
}

void fill_powers(uint64_t *out, uint64_t base, uint64_t step, uint64_t scale, uint64_t count, hipStream_t s)
{
    uint32_t blocks = (uint32_t)((count + 255) / 256);
    hipLaunchKernelGGL(k_fill_powers, dim3(blocks), dim3(256), 0, s, out, base, step, scale, count);
}


// ================================================================ 3-pass LDE
// extendPol for n_ext = 2n (the zkEVM blowup), n = RA * RB with RB = 4096 and
// RA = 2^LA, 6 <= LA <= 12 (n = 2^18 .. 2^24).  DESIGN.md "LDE".
//
// The 2n-point NTT of the zero-padded coset coefficients splits into two
// n-point NTTs (part p = 0, 1):  X[2k + p] = NTT_n(c_i * F_p^i / n)[k] with
// F_p = 7 * omega_2n^p, c = INTT-unscaled coefficients.  With the four-step
// index maps i = jB + RB*jA (evaluations in), c = kA + RA*kB (coefficients)
// and k = k' + RB*k'' (evaluations out):
//   P1 (strided):    INTT over jA for each jB, * omega_n^-(jB kA),
//                    T1[kA*RB + jB]                              read n, write n
//   P2 (contiguous): block kA: INTT over jB -> coefficients kA + RA*kB,
//                    * F_p^c / n, NTT over kB -> k' (both parts),
//                    * omega_n^(kA k'), T2[kA*2RB + 2k' + p]      read n, write 2n
//   P3 (strided):    for each q = 2k' + p: NTT over kA -> k'',
//                    out[q + 2RB*k''] (natural order, in place)  read 2n, write 2n
// 9n element moves = 3x the algorithmic 3n, against 17n for
// INTT + zero-padded NTT as two 3-pass transforms.  Every global access is a
// run of >= 128 bytes: P1 / P3 move 16 consecutive groups per row (LA = 11),
// P2 whole 4096-element blocks.
constexpr int LDE_LB = 12;
constexpr uint64_t LDE_RB = 1ULL << LDE_LB;
constexpr int SP_THREADS = 256;  // strided passes: 64 values per thread, 2 workgroups per CU

struct StridedArgs {
    const uint64_t *src;
    uint64_t src_ld;  // column stride
    uint64_t *dst;
    uint64_t dst_ld;
    uint64_t row_stride;    // distance of consecutive sub-DFT elements, in and out
    const uint64_t *tw_r;   // omega_R^e, e < R (this direction)
    const uint64_t *otw;    // P1: omega_n^-(jB kA) at [kA * RB + jB]; null = none (P3)
    uint32_t canon;         // 1 = canonical output (P3)
    uint32_t ncols;
    uint32_t units;         // workgroups per column
};

// One sub-DFT of size R = 2^LA = 64 * T per group; G = 256 / T groups
// (consecutive positions along the row, the fastest lane index) per workgroup.
//   stage 1: thread (g, t) holds x[t + T*j1], j1 < 64: radix-64 in registers
//            (DIF, twiddles powers of 2 only), * omega_R^(t k1)
//   LDS:     transpose in two 32-bit halves (word k1*ROW + t*G + g; the G
//            pad words per k1 row keep both access patterns conflict-free)
//   stage 2: thread (g, t) holds k1 = t + T*m (m < 64/T), j2 < T:
//            64/T radix-T DFTs -> X[k1 + 64 k2]
template <int LA, bool INV>
__global__ void __launch_bounds__(SP_THREADS) k_lde_strided(StridedArgs a)
{
    constexpr int LT = LA - 6, T = 1 << LT, G = SP_THREADS / T, M = 64 / T;
    constexpr int ROW = T * G + (G < 32 ? G : 0);
    __shared__ uint32_t lds[64 * ROW];
    // columns fastest (the outer-twiddle slice of a unit stays in L2; an
    // XCD-aware order -- each XCD a contiguous range of (column, unit), units
    // fastest -- measured slower, 46.3 vs 48.0 Gelem/s)
    const uint32_t col = blockIdx.x % a.ncols;
    const uint64_t unit = blockIdx.x / a.ncols;
    const uint64_t g0 = unit * G;
    const int tid = threadIdx.x, g = tid % G, t = tid / G;
    const uint64_t rs = a.row_stride;
    const uint64_t *src = a.src + (uint64_t)col * a.src_ld + g0 + g;
    uint64_t v[64];
#pragma unroll
    for (int j1 = 0; j1 < 64; j1++) v[j1] = src[(uint64_t)(t + T * j1) * rs];
    dft_regs<6, INV>(v);
    if constexpr (T > 1) {
#pragma unroll
        for (int r = 1; r < 64; r++) v[r] = gl_mul(v[r], a.tw_r[t * brev_c(r, 6)]);
    }
    // transpose, low words then high words (the low half of v[] takes the
    // new low word as soon as its old one is in LDS)
    const int wb = t * G + g;
#pragma unroll
    for (int r = 0; r < 64; r++) lds[brev_c(r, 6) * ROW + wb] = (uint32_t)v[r];
    __syncthreads();
    uint32_t nl[64];
#pragma unroll
    for (int m = 0; m < M; m++)
#pragma unroll
        for (int j2 = 0; j2 < T; j2++) nl[m * T + j2] = lds[(t + T * m) * ROW + j2 * G + g];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 64; r++) lds[brev_c(r, 6) * ROW + wb] = (uint32_t)(v[r] >> 32);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < M; m++)
#pragma unroll
        for (int j2 = 0; j2 < T; j2++)
            v[m * T + j2] = ((uint64_t)lds[(t + T * m) * ROW + j2 * G + g] << 32) | nl[m * T + j2];
#pragma unroll
    for (int m = 0; m < M; m++) dft_regs<LT, INV>(v + m * T);
    uint64_t *dst = a.dst + (uint64_t)col * a.dst_ld + g0 + g;
    const uint64_t *otw = a.otw ? a.otw + g0 + g : nullptr;
#pragma unroll
    for (int m = 0; m < M; m++) {
#pragma unroll
        for (int r = 0; r < T; r++) {
            const uint64_t k = (uint64_t)(t + T * m) + 64 * (uint64_t)brev_c(r, LT);
            uint64_t x = v[m * T + r];
            if (otw) x = gl_mul(x, otw[k * LDE_RB]);
            dst[k * rs] = a.canon ? gl_canon(x) : x;
        }
    }
}

struct MidArgs {
    const uint64_t *src;  // T1, column stride src_ld
    uint64_t src_ld;
    uint64_t *dst;  // T2 (the output buffer), column stride dst_ld
    uint64_t dst_ld;
    const uint64_t *tw16[2];   // omega_4096^e, e < 4096 (forward, inverse)
    const uint64_t *tw256[2];  // omega_256^e, e < 256
    const uint64_t *fs;        // [p][kA][k]: F_p^(kA + 256 RA k) / n, k < 16
    const uint64_t *twa[2];    // [p][k2 * 256 + t]: F_p^(RA t) omega_4096^(t k2)
    const uint64_t *otw;       // omega_n^(kA k') at [kA * RB + k']
    uint64_t nblk;             // ncols * RA
    uint32_t ncols;
};

constexpr int MID_LDS = 16 * 272;  // u64 per block

// 4096-point DFT of one block by 256 threads, 16 values each, radix 16^3:
// in  thread t holds x[t + 256 j] at v[j];
// out thread t holds X[t + 256 k] at v[brev4(k)].
//   A: DFT over j -> k2, * omega_4096^(t k2), LDS [k2*272 + t]
//   B: thread (j0, k2) = (t & 15, t >> 4) reads j1 < 16 (t = j0 + 16 j1),
//      DFT -> k1, * omega_256^(j0 k1), LDS [j0*257 + k1*16 + k2]
//   C: thread (k2, k1) = (t & 15, t >> 4) reads j0 < 16, DFT -> k0:
//      X[k2 + 16 k1 + 256 k0]
// (pads 272 / 257: conflict-free ds_write_b64 16-lane and ds_read_b64 32-lane groups)
// TA: tw16 is a per-element stage-A table [k2 * 256 + t] (the LDE's
// F_p^(RA t) coset factor folded into omega_4096^(t k2)), else omega_4096^e.
// ZKGPU_LDE_MID_RB=1: P2's butterflies, shift-multiplies and twiddle
// products with the rare corrections behind wave-uniform branches
// (gl_rb.hpp), as the radix-256 pass.  Measured (round 4, A/B twice on one
// box, 3-pass LDE 2^23 -> 2^24 x 100): 42.3 against 49.8 Gelem/s with the
// select form -- the branches split the 200-VGPR kernel's blocks.  Off.
#ifndef ZKGPU_LDE_MID_RB
#define ZKGPU_LDE_MID_RB 0
#endif
__device__ __forceinline__ uint64_t mid_mul(uint64_t a, uint64_t b)
{
    if constexpr (ZKGPU_LDE_MID_RB) return gl_mul_rb(a, b);
    else return gl_mul(a, b);
}

template <bool INV, bool TA>
__device__ __forceinline__ void dft4096_block(uint64_t *v, uint64_t *L, int t, const uint64_t *tw16,
                                              const uint64_t *tw256)
{
    // sched_barrier: keeps the compiler from hoisting the next stage's
    // twiddle loads over the current stage (register pressure)
    dft_regs<4, INV, ZKGPU_LDE_MID_RB>(v);
    if constexpr (TA) {
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = mid_mul(v[r], tw16[(brev_c(r, 4) << 8) + t]);
    } else {
#pragma unroll
        for (int r = 1; r < 16; r++) v[r] = mid_mul(v[r], tw16[t * brev_c(r, 4)]);
    }
#pragma unroll
    for (int r = 0; r < 16; r++) L[brev_c(r, 4) * 272 + t] = v[r];
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    const int lo = t & 15, hi = t >> 4;
#pragma unroll
    for (int j1 = 0; j1 < 16; j1++) v[j1] = L[hi * 272 + lo + 16 * j1];
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    dft_regs<4, INV, ZKGPU_LDE_MID_RB>(v);
#pragma unroll
    for (int r = 1; r < 16; r++) v[r] = mid_mul(v[r], tw256[lo * brev_c(r, 4)]);
#pragma unroll
    for (int r = 0; r < 16; r++) L[lo * 257 + brev_c(r, 4) * 16 + hi] = v[r];
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j0 = 0; j0 < 16; j0++) v[j0] = L[j0 * 257 + hi * 16 + lo];
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    dft_regs<4, INV, ZKGPU_LDE_MID_RB>(v);
}

// P2: one block (kA, column) per workgroup, columns fastest (VGPRs: 16
// values + the 16 coefficients kept for the second part + the first part's
// 16 results, stored with the second's as pairs)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) k_lde_mid(MidArgs a)
{
    __shared__ uint64_t L[MID_LDS];
    const int t = threadIdx.x;
    const uint64_t blk = blockIdx.x;
    const uint32_t col = (uint32_t)(blk % a.ncols);
    const uint64_t kA = blk / a.ncols;
    const uint64_t *src = a.src + (uint64_t)col * a.src_ld + kA * LDE_RB + t;
    uint64_t v[16], c[16];
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = src[256 * j];
    dft4096_block<true, false>(v, L, t, a.tw16[1], a.tw256[1]);
    __builtin_amdgcn_sched_barrier(0);
    // v[brev4(k)] = coefficient kA + RA * (t + 256 k), unscaled
#pragma unroll
    for (int k = 0; k < 16; k++) c[k] = v[brev_c(k, 4)];
    uint64_t *dst = a.dst + (uint64_t)col * a.dst_ld + kA * 2 * LDE_RB + 2 * t;
    const uint64_t *otw = a.otw + kA * LDE_RB + t;
    const uint64_t RA = a.nblk / a.ncols;
    uint64_t z0[16];
    for (int p = 0; p < 2; p++) {
        // coefficient kA + RA (t + 256 k) times F_p^c / n = S_p[kA][k] (block-uniform,
        // scalar loads) * F_p^(RA t) (folded into the stage-A table)
        const uint64_t *S = a.fs + ((uint64_t)p * RA + kA) * 16;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = mid_mul(c[k], S[k]);
        dft4096_block<false, true>(v, L, t, a.twa[p], a.tw256[0]);
        __builtin_amdgcn_sched_barrier(0);
        if (p == 0) {
#pragma unroll
            for (int k = 0; k < 16; k++) z0[k] = v[k];
        }
    }
    // rows 2 (t + 256 k) + {0, 1}: one 16-byte store per pair (whole lines;
    // part-by-part 8-byte stores left half-written lines to the L2)
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint64_t w = otw[256 * k];
        HIP_vector_type<unsigned long long, 2> pr;
        pr.x = mid_mul(z0[brev_c(k, 4)], w);
        pr.y = mid_mul(v[brev_c(k, 4)], w);
        *reinterpret_cast<HIP_vector_type<unsigned long long, 2> *>(dst + 512 * k) = pr;
    }
}

// ---- host side
struct Lde3Tables {
    uint32_t logn = 0;
    uint64_t *pow16[2] = {nullptr, nullptr}, *pow256[2] = {nullptr, nullptr}, *powR[2] = {nullptr, nullptr};
    uint64_t *fs = nullptr, *twa = nullptr;
};

// fs[p][kA][k] = F_p^(kA + 256 RA k) / n
__global__ void k_lde_fs(uint64_t *fs, uint64_t F, uint64_t ninv, uint64_t RA)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= RA * 16) return;
    const uint64_t kA = i >> 4, k = i & 15;
    fs[i] = gl_canon(gl_mul(ninv, gl_pow(F, kA + 256 * RA * k)));
}

// twa[p][k2 * 256 + t] = F_p^(RA t) * omega_4096^(t k2)
__global__ void k_lde_twa(uint64_t *twa, uint64_t F, uint64_t w4096, uint64_t RA)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 4096) return;
    const uint64_t k2 = i >> 8, t = i & 255;
    twa[i] = gl_canon(gl_mul(gl_pow(F, RA * t), gl_pow(w4096, t * k2)));
}
static Lde3Tables g_lde3;

static int lde3_tables(Ctx &ctx, uint32_t logn, hipStream_t s)
{
    Lde3Tables &T = g_lde3;
    if (T.logn == logn) return 0;
    const uint32_t la = logn - LDE_LB;
    const uint64_t RA = 1ULL << la, n = 1ULL << logn;
    auto alloc = [&](uint64_t **p, uint64_t count) -> int {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
        if (hipMalloc((void **)p, count * 8) != hipSuccess) return set_error(ZKGPU_ERR_OOM, "lde tables");
        return 0;
    };
    int rc;
    for (int d = 0; d < 2; d++) {
        const uint64_t w16 = d ? h_inv(h_w(12)) : h_w(12), w256 = d ? h_inv(h_w(8)) : h_w(8),
                       wR = d ? h_inv(h_w(la)) : h_w(la);
        if ((rc = alloc(&T.pow16[d], 4096)) || (rc = alloc(&T.pow256[d], 256)) || (rc = alloc(&T.powR[d], RA)))
            return rc;
        fill_powers(T.pow16[d], w16, 1, 1, 4096, s);
        fill_powers(T.pow256[d], w256, 1, 1, 256, s);
        fill_powers(T.powR[d], wR, 1, 1, RA, s);
    }
    // F_p = 7 * omega_2n^p
    if ((rc = alloc(&T.fs, 2 * RA * 16)) || (rc = alloc(&T.twa, 2 * 4096))) return rc;
    const uint64_t ninv = h_inv(n);
    for (int p = 0; p < 2; p++) {
        const uint64_t F = p ? h_mul(7, h_w(logn + 1)) : 7;
        hipLaunchKernelGGL(k_lde_fs, dim3((uint32_t)((RA * 16 + 255) / 256)), dim3(256), 0, s, T.fs + p * RA * 16, F,
                           ninv, RA);
        hipLaunchKernelGGL(k_lde_twa, dim3(16), dim3(256), 0, s, T.twa + p * 4096, F, h_w(12), RA);
    }
    if ((rc = check_launch("lde tables"))) return rc;
    T.logn = logn;
    return 0;
}

template <int LA>
static void launch_strided(const StridedArgs &a, uint64_t units, int inverse, hipStream_t s)
{
    const dim3 grid((uint32_t)(units * a.ncols));
    if (inverse) hipLaunchKernelGGL((k_lde_strided<LA, true>), grid, dim3(SP_THREADS), 0, s, a);
    else hipLaunchKernelGGL((k_lde_strided<LA, false>), grid, dim3(SP_THREADS), 0, s, a);
}

static void dispatch_strided(uint32_t la, StridedArgs a, uint64_t groups, int inverse, hipStream_t s)
{
    const uint64_t units = groups / (SP_THREADS >> (la - 6));
    a.units = (uint32_t)units;
    switch (la) {
    case 6: launch_strided<6>(a, units, inverse, s); break;
    case 7: launch_strided<7>(a, units, inverse, s); break;
    case 8: launch_strided<8>(a, units, inverse, s); break;
    case 9: launch_strided<9>(a, units, inverse, s); break;
    case 10: launch_strided<10>(a, units, inverse, s); break;
    case 11: launch_strided<11>(a, units, inverse, s); break;
    case 12: launch_strided<12>(a, units, inverse, s); break;
    default: break;
    }
}

// ZKGPU_LDE3=1 selects the 3-pass LDE where it applies (read per call).
// Measured on MI355X (2^23 -> 2^24 x 100, DESIGN.md "LDE"): 35.2 ms against
// 33.5 ms for the 6-pass path with a third of its HBM traffic; both are VALU
// bound, so the 6-pass path stays the default.
bool lde3_supported(uint32_t logn, uint32_t loge)
{
    const char *e = getenv("ZKGPU_LDE3");
    const bool enabled = e && atoi(e) != 0;
    return enabled && loge == logn + 1 && logn >= LDE_LB + 6 && logn <= LDE_LB + 12;
}

static const char *P1_NAMES[13] = {"", "", "", "", "", "", "k_lde_p1<6>", "k_lde_p1<7>", "k_lde_p1<8>", "k_lde_p1<9>",
                                   "k_lde_p1<10>", "k_lde_p1<11>", "k_lde_p1<12>"};
static const char *P3_NAMES[13] = {"", "", "", "", "", "", "k_lde_p3<6>", "k_lde_p3<7>", "k_lde_p3<8>", "k_lde_p3<9>",
                                   "k_lde_p3<10>", "k_lde_p3<11>", "k_lde_p3<12>"};

// out (2n rows, column stride ld_out >= 2n) = extendPol(in); t1: n words per column
int lde3_columns(Ctx &ctx, uint64_t *out, uint64_t ld_out, const uint64_t *in, uint64_t ld_in, uint64_t *t1,
                 uint32_t logn, uint64_t ncols, hipStream_t s)
{
    if (logn < LDE_LB + 6 || logn > LDE_LB + 12) return set_error(ZKGPU_ERR_ARG, "lde3: unsupported size 2^%u", logn);
    if (ncols == 0) return 0;
    int rc;
    if ((rc = lde3_tables(ctx, logn, s))) return rc;
    const uint32_t la = logn - LDE_LB;
    const uint64_t n = 1ULL << logn, RA = 1ULL << la;
    const uint64_t *otw_inv = otw_table(ctx, 1, logn, la, s), *otw_fwd = otw_table(ctx, 0, logn, la, s);
    if (!otw_inv || !otw_fwd) return set_error(ZKGPU_ERR_OOM, "lde3: twiddle tables");
    // at most 65535 columns and 2^31 workgroups per launch
    const uint64_t cmax = std::min<uint64_t>(65535, (1ULL << 31) / (2 * LDE_RB));
    for (uint64_t c0 = 0; c0 < ncols; c0 += cmax) {
        const uint32_t nc = (uint32_t)std::min<uint64_t>(cmax, ncols - c0);
        StridedArgs p1;
        p1.src = in + c0 * ld_in;
        p1.src_ld = ld_in;
        p1.dst = t1;
        p1.dst_ld = n;
        p1.row_stride = LDE_RB;
        p1.tw_r = g_lde3.powR[1];
        p1.otw = otw_inv;
        p1.canon = 0;
        p1.ncols = nc;
        prof_begin(s);
        dispatch_strided(la, p1, LDE_RB, 1, s);
        prof_end(P1_NAMES[la], 16.0 * (double)n * nc, s);
        MidArgs m;
        m.src = t1;
        m.src_ld = n;
        m.dst = out + c0 * ld_out;
        m.dst_ld = ld_out;
        for (int d = 0; d < 2; d++) {
            m.tw16[d] = g_lde3.pow16[d];
            m.tw256[d] = g_lde3.pow256[d];
            m.twa[d] = g_lde3.twa + d * 4096;
        }
        m.fs = g_lde3.fs;
        m.otw = otw_fwd;
        m.nblk = RA * nc;
        m.ncols = nc;
        prof_begin(s);
        hipLaunchKernelGGL(k_lde_mid, dim3((uint32_t)m.nblk), dim3(256), 0, s, m);
        prof_end("k_lde_mid", 24.0 * (double)n * nc, s);
        StridedArgs p3;
        p3.src = out + c0 * ld_out;
        p3.src_ld = ld_out;
        p3.dst = out + c0 * ld_out;
        p3.dst_ld = ld_out;
        p3.row_stride = 2 * LDE_RB;
        p3.tw_r = g_lde3.powR[0];
        p3.otw = nullptr;
        p3.canon = 1;
        p3.ncols = nc;
        prof_begin(s);
        dispatch_strided(la, p3, 2 * LDE_RB, 0, s);
        prof_end(P3_NAMES[la], 32.0 * (double)n * nc, s);
    }
    return check_launch("lde3");
}

}  // namespace zk
