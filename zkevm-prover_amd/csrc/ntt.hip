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
#include "gl_device.hpp"
#include "zkgpu_internal.hpp"

namespace zk {

// ---------------------------------------------------------------- tables
// k_fill_powers: out[i] = scale * base^(i * step) for i < count
__global__ void k_fill_powers(uint64_t *out, uint64_t base, uint64_t step, uint64_t scale, uint64_t count)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint64_t b = gl_pow(base, step);
    out[i] = gl_mul(scale, gl_pow(b, i));
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
    uint64_t *dst;
    uint64_t dst_ld;
    const uint64_t *rt_small;  // omega_4096^k, k < 2048, for this direction
    const uint64_t *tw_lo;     // big twiddles, this direction
    const uint64_t *tw_hi;
    const uint64_t *post_lo;  // post-scale (last pass), may be null
    const uint64_t *post_hi;
    uint64_t post_scale;  // applied when post_lo == null and != 1
    uint32_t post_bits;
    uint32_t logn;
    uint32_t logm;      // block size before this pass (first pass: logn)
    uint32_t last;      // 1 = last pass (digit-reversed scatter)
    uint32_t npass;
    uint32_t rbits[NTT_MAX_PASSES];
    uint32_t pass_idx;  // index of this pass
};

constexpr int PASS_THREADS = 256;
constexpr int GROUPS = 16;

// DIF radix-2 over LDS: 16 groups x R elements, element (j, g) at lds[j*16+g].
template <int LOGR>
__device__ __forceinline__ void dif_lds(uint64_t *lds, const uint64_t *tw)
{
    constexpr int R = 1 << LOGR;
    constexpr int NB = GROUPS * R / 2;
#pragma unroll
    for (int lh = LOGR - 1; lh >= 0; lh--) {
        const int h = 1 << lh;
        __syncthreads();
        for (int bi = threadIdx.x; bi < NB; bi += PASS_THREADS) {
            int g = bi & 15;
            int b = bi >> 4;
            int pos = b & (h - 1);
            int i0 = ((b >> lh) << (lh + 1)) + pos;
            int i1 = i0 + h;
            uint64_t a = lds[i0 * 16 + g];
            uint64_t c = lds[i1 * 16 + g];
            lds[i0 * 16 + g] = gl_add(a, c);
            uint64_t d = gl_sub(a, c);
            lds[i1 * 16 + g] = (pos == 0) ? d : gl_mul(d, tw[pos << (LOGR - 1 - lh)]);
        }
    }
    __syncthreads();
}

template <int LOGR>
__global__ void __launch_bounds__(PASS_THREADS) k_ntt_pass(PassArgs a)
{
    constexpr int R = 1 << LOGR;
    __shared__ uint64_t lds[GROUPS * R];
    __shared__ uint64_t tw[R / 2];
    const uint32_t col = blockIdx.y;
    const uint64_t *src = a.src + (uint64_t)col * a.src_ld;
    uint64_t *dst = a.dst + (uint64_t)col * a.dst_ld;
    const int tid = threadIdx.x;

    for (int k = tid; k < R / 2; k += PASS_THREADS) tw[k] = a.rt_small[k << (12 - LOGR)];

    const uint64_t u = blockIdx.x;
    if (!a.last) {
        // ---- first / middle pass: in-place layout
        const uint32_t logmp = a.logm - LOGR;  // log2 m'
        const uint64_t mp = 1ULL << logmp;
        const uint64_t groups_per_blk = mp >> 4;
        const uint64_t blk = u / groups_per_blk;
        const uint64_t j0 = (u % groups_per_blk) << 4;
        const uint64_t base = (blk << a.logm) + j0;
        const int g = tid & 15;
#pragma unroll
        for (int it = 0; it < R / 16; it++) {
            int j = (tid >> 4) + 16 * it;
            uint64_t pos = base + ((uint64_t)j << logmp) + g;
            uint64_t v = pos < a.src_valid ? gl_canon(src[pos]) : 0;
            lds[j * 16 + g] = v;
        }
        dif_lds<LOGR>(lds, tw);
        const uint32_t tshift = TW_MAX_LOG - a.logm;
        const uint64_t jp = j0 + g;
#pragma unroll
        for (int it = 0; it < R / 16; it++) {
            int k = (tid >> 4) + 16 * it;
            uint64_t v = lds[bitrev_u32(k, LOGR) * 16 + g];
            uint64_t e = (jp * (uint64_t)k) << tshift;
            if (e) v = gl_mul(v, tw_big(a.tw_lo, a.tw_hi, e));
            dst[base + ((uint64_t)k << logmp) + g] = v;
        }
    } else {
        // ---- last pass: 16 blocks with consecutive leading digit k_1
        // blk = k_1 * S + rest, S = n / (r_1 * R)
        const uint32_t r1b = a.rbits[0];
        const uint32_t logS = a.logn - r1b - LOGR;
        const uint64_t S = 1ULL << logS;
        const uint64_t rest = u & (S - 1);
        const uint64_t k1g = u >> logS;
        // reversed digits of rest (radices rbits[1..npass-2])
        uint64_t rrev = 0;
        {
            // rest = sum_{i=1..npass-2} k_i * prod_{l>i} r_l (k_1 of rest most significant);
            // rrev = sum_i k_i * prod_{1<=l<i} r_l  (mixed-radix digit reversal)
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
        // load 16 blocks x R contiguous elements
        for (int e = tid; e < GROUPS * R; e += PASS_THREADS) {
            int g = e >> LOGR;
            int t = e & (R - 1);
            uint64_t blk = ((k1g * 16 + g) << logS) + rest;
            uint64_t pos = (blk << LOGR) + t;
            uint64_t v = pos < a.src_valid ? gl_canon(src[pos]) : 0;
            lds[t * 16 + g] = v;
        }
        dif_lds<LOGR>(lds, tw);
        const int g = tid & 15;
        const uint64_t xbase = (k1g * 16 + g) + (rrev << r1b);
        const uint32_t lognr = a.logn - LOGR;
#pragma unroll
        for (int it = 0; it < R / 16; it++) {
            int k = (tid >> 4) + 16 * it;
            uint64_t v = lds[bitrev_u32(k, LOGR) * 16 + g];
            uint64_t x = xbase + ((uint64_t)k << lognr);
            if (a.post_lo) {
                uint64_t f = gl_mul(a.post_lo[x & ((1ULL << a.post_bits) - 1)], a.post_hi[x >> a.post_bits]);
                v = gl_mul(v, f);
            } else if (a.post_scale != 1) {
                v = gl_mul(v, a.post_scale);
            }
            dst[x] = v;
        }
    }
}

// ---------------------------------------------------------------- small NTT
// one workgroup per column, whole column (n <= 4096) in LDS
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
    for (uint32_t i = threadIdx.x; i < n; i += PASS_THREADS) lds[i] = i < a.src_valid ? gl_canon(src[i]) : 0;
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
        dst[k] = v;
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

// ---------------------------------------------------------------- host side
static const char *PASS_NAMES[9] = {"", "", "", "", "k_ntt_pass<4>", "k_ntt_pass<5>",
                                     "k_ntt_pass<6>", "k_ntt_pass<7>", "k_ntt_pass<8>"};

static void split_radix(uint32_t logn, uint32_t *npass, uint32_t rbits[NTT_MAX_PASSES])
{
    uint32_t P = (logn + 7) / 8;
    *npass = P;
    uint32_t base = logn / P, extra = logn % P;
    // larger radices last (the last pass reads contiguous runs of R)
    for (uint32_t i = 0; i < P; i++) rbits[i] = base + (i >= P - extra ? 1 : 0);
}

template <int LOGR>
static void launch_pass(const PassArgs &a, uint64_t ncols, hipStream_t s)
{
    uint64_t units = (1ULL << (a.logn - LOGR)) / 16;
    dim3 grid((uint32_t)units, (uint32_t)ncols);
    hipLaunchKernelGGL(k_ntt_pass<LOGR>, grid, dim3(PASS_THREADS), 0, s, a);
}

static void dispatch_pass(uint32_t logr, const PassArgs &a, uint64_t ncols, hipStream_t s)
{
    switch (logr) {
    case 4: launch_pass<4>(a, ncols, s); break;
    case 5: launch_pass<5>(a, ncols, s); break;
    case 6: launch_pass<6>(a, ncols, s); break;
    case 7: launch_pass<7>(a, ncols, s); break;
    case 8: launch_pass<8>(a, ncols, s); break;
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
                const uint64_t *post_hi, uint32_t post_bits, uint64_t post_scale, hipStream_t s)
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
    a.rt_small = ctx.rt_small[d];
    a.tw_lo = ctx.tw_lo[d];
    a.tw_hi = ctx.tw_hi[d];
    a.logn = logn;
    split_radix(logn, &a.npass, a.rbits);
    uint32_t logm = logn;
    for (uint32_t p = 0; p < a.npass; p++) {
        a.pass_idx = p;
        a.logm = logm;
        a.last = (p == a.npass - 1);
        a.post_lo = a.last ? post_lo : nullptr;
        a.post_hi = a.last ? post_hi : nullptr;
        a.post_bits = post_bits;
        a.post_scale = a.last ? post_scale : 1;
        if (p == 0) {
            a.src = src;
            a.src_ld = src_ld;
            a.src_valid = src_valid;
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
        for (uint64_t c0 = 0; c0 < ncols; c0 += 65535) {
            uint64_t nc = ncols - c0 < 65535 ? ncols - c0 : 65535;
            PassArgs b = a;
            b.src = a.src + c0 * a.src_ld;
            b.dst = a.dst + c0 * a.dst_ld;
            prof_begin(s);
            dispatch_pass(a.rbits[p], b, nc, s);
            prof_end(PASS_NAMES[a.rbits[p]], 8.0 * (double)(nread + n) * (double)nc, s);
        }
        logm -= a.rbits[p];
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

}  // namespace zk
