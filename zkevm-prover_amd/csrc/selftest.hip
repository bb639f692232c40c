// Arithmetic self-test hook for the rare-branch field helpers (csrc/gl_rb.hpp,
// gl_add_rb / gl_sub_rb in csrc/gl_device.hpp, the Poseidon S-box products of
// csrc/poseidon_perm.hpp) and the shift-multiplies mul2e / mul2e_rb for every
// exponent.  Each helper takes its final correction behind a wave-uniform
// branch (the lane mask of the correction's own compare), so a random input
// almost never reaches it: the parity tests (tests/test_gpu_rb.py) feed inputs
// crafted to force the correction, in every lane of a wave and in exactly one
// lane of an otherwise ordinary wave, and compare with big integers.  Test
// infrastructure inside the product library: nothing on the proof path calls
// it.  Reference semantics: the Goldilocks field ops used at starks.cpp:53.
#include <utility>

#include "gl_device.hpp"
#include "gl_rb.hpp"
#include "poseidon_perm.hpp"
#include "zkgpu_internal.hpp"

namespace zk {

template <int... Es>
__device__ __forceinline__ uint64_t mul2e_any(int e, uint64_t x, bool rb, std::integer_sequence<int, Es...>)
{
    uint64_t r = 0;
    (void)((e == Es ? (r = rb ? mul2e_rb<Es>(x) : mul2e<Es>(x), true) : false) || ...);
    return r;
}

__global__ void k_field_selftest_rb(uint64_t *out, const uint64_t *a, const uint64_t *b, const uint64_t *c, uint64_t n,
                                    int op, int e)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // every lane of the last wave runs the op (inactive lanes on a clamped
    // index) so the ballots see whole waves, as in the product kernels
    const uint64_t j = i < n ? i : n - 1;
    const uint64_t x = a[j], y = b[j];
    uint64_t r = 0;
    switch (op) {
    case 0: r = gl_add_rb(x, y); break;
    case 1: r = gl_sub_rb(x, y); break;
    case 2: r = gl_mul_rb(x, y); break;
    case 3: r = gl_reduce128_rb(x, y); break;
    case 4: r = gl_reduce96_small_rb(x, (uint32_t)y); break;
    case 5: {
        Dot3 d;
        d.A0 = x;
        d.A1 = y;
        d.A2 = c[j];
        r = dot3_fin_rb(d);
        break;
    }
    case 6: r = mul2e_any(e, x, true, std::make_integer_sequence<int, 192>{}); break;
    case 7: r = mul2e_any(e, x, false, std::make_integer_sequence<int, 192>{}); break;
    case 8: r = pow7(x); break;  // the Poseidon S-box (gl_sqr3 + gl_mul_rb)
    case 9: r = gl_sqr3(x); break;
    case 10: r = gl_reduce128(x, y); break;
    case 11: {
        Dot3 d;
        d.A0 = x;
        d.A1 = y;
        d.A2 = c[j];
        r = d.fin();
        break;
    }
    default: break;
    }
    if (i < n) out[i] = gl_canon(r);
}

}  // namespace zk

using namespace zk;

extern "C" int zkgpu_gl_field_selftest_rb_dev(uint64_t *out, const uint64_t *a, const uint64_t *b, const uint64_t *c,
                                               uint64_t n, int op, int e)
{
    if (!ctx().ready) return set_error(ZKGPU_ERR_INIT, "zkgpu_init() not called");
    if (op < 0 || op > 11) return set_error(ZKGPU_ERR_ARG, "field_selftest_rb: unknown op %d", op);
    if ((op == 6 || op == 7) && (e < 0 || e >= 192)) return set_error(ZKGPU_ERR_ARG, "field_selftest_rb: e %d", e);
    if ((op == 5 || op == 11) && !c) return set_error(ZKGPU_ERR_ARG, "field_selftest_rb: op %d needs c", op);
    if (!n) return 0;
    hipLaunchKernelGGL(k_field_selftest_rb, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, ctx().stream, out, a, b,
                       c, n, op, e);
    return check_launch("k_field_selftest_rb");
}
