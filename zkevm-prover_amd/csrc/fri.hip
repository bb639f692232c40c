// FRI fold and group-transpose kernels for gfx950.
//
// Replaces the fold loop of FRIProve::prove (friProve.cpp:44-108) and
// FRIProve::getTransposed (friProve.cpp:252-270).
//   out[g] = Horner_{special_x}( INTT_nX(pol[i*2^out_bits + g])_i * (shiftInv * w(pol_bits)^-g)^i )
// One thread per output group g: the nX strided ext reads are coalesced
// across consecutive g, the nX-point INTT runs in registers (radix-2, fully
// unrolled per nX), the 1/nX scale is folded into the power sequence.
#include "gl_device.hpp"
#include "zkgpu_internal.hpp"

namespace zk {

__device__ __forceinline__ uint32_t brev(uint32_t x, uint32_t bits)
{
    return bits == 0 ? 0 : (__builtin_bitreverse32(x) >> (32 - bits));
}

// Groups [g0, g0 + n_local) of the fold; element i of local group gl at
// pol + 3 (i istride + gl gstride): the whole polynomial (g0 = 0, istride =
// 2^out_bits, gstride = 1) or a block of its getTransposed rows (istride 1,
// gstride nX: the sharded prover's first fold, host/sharded_starks.hpp).
template <int LOGNX>
__global__ void __launch_bounds__(256) k_fri_fold(uint64_t *out, const uint64_t *__restrict__ pol, uint32_t pol_bits,
                                                 uint32_t out_bits, gl3 sx, uint64_t shift_inv,
                                                 const uint64_t *rt_inv, const uint64_t *tw_lo_inv,
                                                 const uint64_t *tw_hi_inv, uint64_t g0, uint64_t n_local,
                                                 uint64_t istride, uint64_t gstride)
{
    constexpr int NX = 1 << LOGNX;
    const uint64_t gl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gl >= n_local) return;
    const uint64_t g = g0 + gl;
    gl3 v[NX];
    // bit-reversed load -> DIT
#pragma unroll
    for (int i = 0; i < NX; i++) {
        const uint64_t *p = pol + 3 * ((uint64_t)i * istride + gl * gstride);
        int r = brev(i, LOGNX);
        v[r].v[0] = p[0];
        v[r].v[1] = p[1];
        v[r].v[2] = p[2];
    }
#pragma unroll
    for (int s = 1; s <= LOGNX; s++) {
        const int half = 1 << (s - 1);
#pragma unroll
        for (int b = 0; b < NX; b += 2 * half) {
#pragma unroll
            for (int i = 0; i < half; i++) {
                // omega_{2 half}^{-i} = omega_4096^{-(i * 4096/(2 half))}
                gl3 t = v[b + i + half];
                if (i) t = gl3_mul1(t, rt_inv[i << (12 - s)]);
                gl3 a = v[b + i];
                v[b + i] = gl3_add(a, t);
                v[b + i + half] = gl3_sub(a, t);
            }
        }
    }
    // c_i *= (1/nX) * (shiftInv * w^-g)^i ;  w^-g = omega_{2^28}^{-(g << (28 - pol_bits))}
    uint64_t e = g << (TW_MAX_LOG - pol_bits);
    uint64_t wg = gl_mul(tw_lo_inv[e & (TW_LEVEL_SIZE - 1)], tw_hi_inv[e >> TW_LEVEL_BITS]);
    uint64_t sinv = gl_mul(shift_inv, wg);  // shiftInv * w^-g
    uint64_t r = 1;
    // 1/nX scale
    const uint64_t nx_inv = ZK_P - ((ZK_P - 1) >> LOGNX);  // (1/nX) mod p = p - (p-1)/nX
#pragma unroll
    for (int i = 0; i < NX; i++) {
        v[i] = gl3_mul1(v[i], gl_mul(r, nx_inv));
        r = gl_mul(r, sinv);
    }
    gl3 acc = v[NX - 1];
#pragma unroll
    for (int i = NX - 2; i >= 0; i--) acc = gl3_add(gl3_mul(acc, sx), v[i]);
    uint64_t *o = out + 3 * gl;
    o[0] = gl_canon(acc.v[0]);
    o[1] = gl_canon(acc.v[1]);
    o[2] = gl_canon(acc.v[2]);
}

__global__ void k_fri_transpose(uint64_t *aux, const uint64_t *pol, uint64_t w, uint64_t h)
{
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w * h) return;
    // destination-ordered: di = i*h + j  <-  fi = j*w + i
    uint64_t i = t / h, j = t % h;
    uint64_t fi = j * w + i;
    aux[3 * t + 0] = pol[3 * fi + 0];
    aux[3 * t + 1] = pol[3 * fi + 1];
    aux[3 * t + 2] = pol[3 * fi + 2];
}

template <int L>
static void launch_fold(uint64_t *out, const uint64_t *pol, uint32_t pol_bits, uint32_t out_bits, gl3 sx,
                        uint64_t sinv, uint64_t g0, uint64_t n_local, bool rows, hipStream_t s)
{
    Ctx &c = ctx();
    const uint64_t istride = rows ? 1 : (1ULL << out_bits), gstride = rows ? (1ULL << L) : 1;
    uint32_t blocks = (uint32_t)((n_local + 255) / 256);
    prof_begin(s);
    hipLaunchKernelGGL(k_fri_fold<L>, dim3(blocks), dim3(256), 0, s, out, pol, pol_bits, out_bits, sx, sinv,
                       c.rt_small[1], c.tw_lo[1], c.tw_hi[1], g0, n_local, istride, gstride);
    prof_end("k_fri_fold", 24.0 * (double)(n_local << L) + 24.0 * (double)n_local, s);
}

// groups [g0, g0 + n_local) of the fold 2^pol_bits -> 2^out_bits; rows:
// `pol` holds those groups' getTransposed rows (nX elements each) instead of
// the whole polynomial
static int fri_fold_any(uint64_t *out, const uint64_t *pol, uint32_t pol_bits, uint32_t out_bits,
                        const uint64_t sx_h[3], uint64_t shift_inv, uint64_t g0, uint64_t n_local, bool rows,
                        hipStream_t s)
{
    if (out_bits > pol_bits || pol_bits > TW_MAX_LOG)
        return set_error(ZKGPU_ERR_ARG, "fri_fold: bad bits %u -> %u", pol_bits, out_bits);
    if (g0 + n_local > (1ULL << out_bits) || g0 + n_local < g0)
        return set_error(ZKGPU_ERR_ARG, "fri_fold: groups [%llu, +%llu) outside the 2^%u outputs",
                         (unsigned long long)g0, (unsigned long long)n_local, out_bits);
    if (!n_local) return 0;
    gl3 sx{{sx_h[0] % ZK_P, sx_h[1] % ZK_P, sx_h[2] % ZK_P}};
    uint64_t sinv = shift_inv % ZK_P;
    switch (pol_bits - out_bits) {
    case 0: launch_fold<0>(out, pol, pol_bits, out_bits, sx, sinv, g0, n_local, rows, s); break;
    case 1: launch_fold<1>(out, pol, pol_bits, out_bits, sx, sinv, g0, n_local, rows, s); break;
    case 2: launch_fold<2>(out, pol, pol_bits, out_bits, sx, sinv, g0, n_local, rows, s); break;
    case 3: launch_fold<3>(out, pol, pol_bits, out_bits, sx, sinv, g0, n_local, rows, s); break;
    case 4: launch_fold<4>(out, pol, pol_bits, out_bits, sx, sinv, g0, n_local, rows, s); break;
    case 5: launch_fold<5>(out, pol, pol_bits, out_bits, sx, sinv, g0, n_local, rows, s); break;
    default: return set_error(ZKGPU_ERR_ARG, "fri_fold: reduction of %u bits > 5 unsupported", pol_bits - out_bits);
    }
    return check_launch("k_fri_fold");
}

int fri_fold(uint64_t *out, const uint64_t *pol, uint32_t pol_bits, uint32_t out_bits, const uint64_t sx_h[3],
             uint64_t shift_inv, hipStream_t s)
{
    return fri_fold_any(out, pol, pol_bits, out_bits, sx_h, shift_inv, 0, 1ULL << out_bits, false, s);
}

int fri_fold_rows(uint64_t *out, const uint64_t *rows, uint64_t g0, uint64_t n_local, uint32_t pol_bits,
                  uint32_t out_bits, const uint64_t sx_h[3], uint64_t shift_inv, hipStream_t s)
{
    return fri_fold_any(out, rows, pol_bits, out_bits, sx_h, shift_inv, g0, n_local, true, s);
}

int fri_transpose(uint64_t *aux, const uint64_t *pol, uint64_t degree, uint32_t tbits, hipStream_t s)
{
    uint64_t w = 1ULL << tbits;
    if (degree % w) return set_error(ZKGPU_ERR_ARG, "fri_transpose: degree not a multiple of 2^%u", tbits);
    uint64_t h = degree / w;
    uint32_t blocks = (uint32_t)((degree + 255) / 256);
    if (!degree) return 0;
    hipLaunchKernelGGL(k_fri_transpose, dim3(blocks), dim3(256), 0, s, aux, pol, w, h);
    return check_launch("k_fri_transpose");
}

}  // namespace zk
