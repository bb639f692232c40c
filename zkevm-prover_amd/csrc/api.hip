// libzkgpu C-ABI (include/zkgpu.h): context, tables, host-pointer drop-ins
// and device-resident entry points.  All bulk arithmetic runs in the HIP
// kernels of ntt.hip / poseidon.hip / fri.hip; the host only stages buffers
// and computes a handful of scalar constants (roots, inverses).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "gl_device.hpp"
#include "zkgpu_internal.hpp"
#include "poseidon_gl_constants.h"
#include "poseidon_gl_sparse.h"

namespace zk {

int upload_poseidon_constants(Ctx &c);

static Ctx g_ctx;
static thread_local char g_err[512] = "";

Ctx &ctx() { return g_ctx; }

int set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int check_hip(hipError_t e, const char *what)
{
    if (e != hipSuccess) return set_error(ZKGPU_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return ZKGPU_OK;
}

int check_launch(const char *what) { return check_hip(hipGetLastError(), what); }

uint64_t *workspace(int i, size_t bytes)
{
    Workspace &w = g_ctx.ws[i];
    if (w.bytes >= bytes) return (uint64_t *)w.ptr;
    if (w.ptr) {
        (void)hipStreamSynchronize(g_ctx.stream);
        (void)hipFree(w.ptr);
        w.ptr = nullptr;
        w.bytes = 0;
    }
    if (hipMalloc(&w.ptr, bytes) != hipSuccess) {
        w.ptr = nullptr;
        set_error(ZKGPU_ERR_OOM, "workspace %d: hipMalloc(%zu) failed", i, bytes);
        return nullptr;
    }
    w.bytes = bytes;
    return (uint64_t *)w.ptr;
}

// ---- host scalar field (setup constants only)
static const uint64_t HP = 0xFFFFFFFF00000001ULL;
// (a b) mod p by the Goldilocks folding 2^64 = 2^32 - 1, 2^96 = -1 (no 128-bit
// division: the expression kernels' limb tables take ~10^5 of these per proof)
uint64_t h_mul(uint64_t a, uint64_t b)
{
    const unsigned __int128 x = (unsigned __int128)a * b;
    const uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64), eps = 0xFFFFFFFFULL;
    const uint64_t hh = hi >> 32, hl = hi & eps;
    uint64_t t0 = lo - hh;
    if (lo < hh) t0 -= eps;  // borrow: 2^64 == eps
    const uint64_t t1 = (hl << 32) - hl;
    uint64_t r = t0 + t1;
    if (r < t1) r += eps;  // carry: no second one
    return r >= HP ? r - HP : r;
}
uint64_t h_pow(uint64_t a, uint64_t e)
{
    uint64_t r = 1;
    a %= HP;
    while (e) {
        if (e & 1) r = h_mul(r, a);
        a = h_mul(a, a);
        e >>= 1;
    }
    return r;
}
uint64_t h_inv(uint64_t a) { return h_pow(a, HP - 2); }
uint64_t h_w(uint32_t n)
{
    uint64_t w = 7277203076849721926ULL;  // W[32]
    for (uint32_t i = n; i < 32; i++) w = h_mul(w, w);
    return w;
}

static int alloc_dev(uint64_t **p, size_t n)
{
    if (hipMalloc((void **)p, n * sizeof(uint64_t)) != hipSuccess)
        return set_error(ZKGPU_ERR_OOM, "hipMalloc(%zu) failed", n * sizeof(uint64_t));
    return 0;
}

// LDE post-scale tables: factor(k) = 1/n * 7^k = lo[k & 4095] * hi[k >> 12]
static int ensure_post_tables(uint32_t logn)
{
    Ctx &c = g_ctx;
    if (c.post_lo && c.post_logn == logn) return 0;
    if (c.post_lo) {
        (void)hipStreamSynchronize(c.stream);
        (void)hipFree(c.post_lo);
        (void)hipFree(c.post_hi);
        c.post_lo = c.post_hi = nullptr;
    }
    uint64_t n = 1ULL << logn;
    uint64_t nlo = 1ULL << POST_BITS;
    uint64_t nhi = n > nlo ? n >> POST_BITS : 1;
    int rc;
    if ((rc = alloc_dev(&c.post_lo, nlo)) || (rc = alloc_dev(&c.post_hi, nhi))) return rc;
    fill_powers(c.post_lo, 7, 1, 1, nlo, c.stream);
    fill_powers(c.post_hi, 7, nlo, h_inv(n), nhi, c.stream);
    c.post_logn = logn;
    return check_launch("post tables");
}

static int require_init()
{
    if (!g_ctx.ready) return set_error(ZKGPU_ERR_INIT, "zkgpu_init() not called");
    return 0;
}

static bool is_pow2(uint64_t n) { return n && !(n & (n - 1)); }
static uint32_t log2u(uint64_t n)
{
    uint32_t l = 0;
    while ((1ULL << l) < n) l++;
    return l;
}

// Columns per extend_pol batch: the batch's coefficients (n words per
// column) and, on the 6-pass path, its 2n-row scratch live in grow-only
// workspaces, so the batch bounds that memory -- 2^31 words (16 GiB) of
// scratch.  (Batches of 32 columns
// at 2^24 rows measured 2-3 % slower than one batch of 100: 51.9 vs 53.5
// Gelem/s, the same box.)
static uint64_t g_lde_batch_max = 0;  // zkgpu_set_lde_batch_cols (0: the default)
static uint64_t lde_batch_cols(uint64_t n_ext, uint64_t ncols)
{
    uint64_t batch = std::max<uint64_t>(1, (1ULL << 31) / (n_ext ? n_ext : 1));
    if (g_lde_batch_max && g_lde_batch_max < batch) batch = g_lde_batch_max;
    return batch < ncols ? batch : ncols;
}

static uint64_t lde_workspace_bytes(uint64_t n, uint64_t n_ext, uint64_t ncols)
{
    const uint64_t b = lde_batch_cols(n_ext, ncols);
    return b * n * 8 + (lde3_supported(log2u(n), log2u(n_ext)) ? 0 : b * n_ext * 8);
}

// device LDE on column-major buffers
static int extend_pol_dev(uint64_t *out, uint64_t ld_out, const uint64_t *in, uint64_t ld_in, uint64_t n_ext,
                          uint64_t n, uint64_t ncols)
{
    if (!ncols || !n) return 0;
    if (!is_pow2(n) || !is_pow2(n_ext) || n_ext < n)
        return set_error(ZKGPU_ERR_ARG, "extend_pol: sizes must be powers of two with n_ext >= n");
    uint32_t logn = log2u(n), loge = log2u(n_ext);
    if (loge > TW_MAX_LOG) return set_error(ZKGPU_ERR_ARG, "extend_pol: n_ext > 2^%u", TW_MAX_LOG);
    int rc;
    if ((rc = ensure_post_tables(logn))) return rc;
    Ctx &c = g_ctx;
    const uint64_t batch = lde_batch_cols(n_ext, ncols);
    uint64_t *coef = workspace(0, batch * n * sizeof(uint64_t));
    if (!coef) return ZKGPU_ERR_OOM;
    if (lde3_supported(logn, loge)) {
        for (uint64_t c0 = 0; c0 < ncols; c0 += batch) {
            const uint64_t nc = ncols - c0 < batch ? ncols - c0 : batch;
            if ((rc = lde3_columns(c, out + c0 * ld_out, ld_out, in + c0 * ld_in, ld_in, coef, logn, nc, c.stream)))
                return rc;
        }
        return 0;
    }
    uint64_t *tmp = workspace(1, batch * n_ext * sizeof(uint64_t));
    if (!tmp) return ZKGPU_ERR_OOM;
    uint32_t post_bits = logn < POST_BITS ? logn : POST_BITS;
    for (uint64_t c0 = 0; c0 < ncols; c0 += batch) {
        uint64_t nc = ncols - c0 < batch ? ncols - c0 : batch;
        // coefficients * 7^k / n
        if ((rc = ntt_columns(c, coef, n, in + c0 * ld_in, ld_in, n, tmp, n, logn, nc, 1, c.post_lo, c.post_hi,
                              post_bits, 7, 1, c.stream)))
            return rc;
        // evaluations on the extended domain (zero padding = predicated loads)
        if ((rc = ntt_columns(c, out + c0 * ld_out, ld_out, coef, n, n, tmp, n_ext, loge, nc, 0, nullptr, nullptr, 0,
                              1, 1, c.stream)))
            return rc;
    }
    return 0;
}

static int ntt_dev(uint64_t *dst, uint64_t ld_dst, const uint64_t *src, uint64_t ld_src, uint64_t n, uint64_t ncols,
                   int inverse)
{
    if (!ncols || !n) return 0;
    if (!is_pow2(n)) return set_error(ZKGPU_ERR_ARG, "ntt: n must be a power of two");
    uint32_t logn = log2u(n);
    if (logn > TW_MAX_LOG) return set_error(ZKGPU_ERR_ARG, "ntt: n > 2^%u", TW_MAX_LOG);
    Ctx &c = g_ctx;
    uint64_t *tmp = nullptr;
    if (logn > 12) {
        tmp = workspace(1, ncols * n * sizeof(uint64_t));
        if (!tmp) return ZKGPU_ERR_OOM;
    }
    uint64_t scale = inverse ? h_inv(n) : 1;
    return ntt_columns(c, dst, ld_dst, src, ld_src, n, tmp, n, logn, ncols, inverse, nullptr, nullptr, 0, 1, scale,
                       c.stream);
}

__global__ void k_field_selftest(uint64_t *out, const uint64_t *a, const uint64_t *b, uint64_t n, int op)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (op == 9) {
        gl3 x{{a[3 * i], a[3 * i + 1], a[3 * i + 2]}}, y{{b[3 * i], b[3 * i + 1], b[3 * i + 2]}};
        gl3 r = gl3_canon(gl3_mul(x, y));
        out[3 * i] = r.v[0];
        out[3 * i + 1] = r.v[1];
        out[3 * i + 2] = r.v[2];
        return;
    }
    uint64_t x = a[i], y = b[i], r = 0;
    switch (op) {
    case 0: r = gl_add(x, y); break;
    case 1: r = gl_sub(x, y); break;
    case 2: r = gl_mul(x, y); break;
    case 3: r = gl_neg(x); break;
    case 4: r = mul2e<12>(x); break;
    case 5: r = mul2e<48>(x); break;
    case 6: r = mul2e<84>(x); break;
    case 7: r = mul2e<100>(x); break;
    case 8: {
        uint64_t x2 = gl_mul(x, x), x3 = gl_mul(x2, x), x4 = gl_mul(x2, x2);
        r = gl_mul(x3, x4);
        break;
    }
    default: break;
    }
    out[i] = gl_canon(r);
}

}  // namespace zk

using namespace zk;

extern "C" {

int zkgpu_gl_field_selftest_dev(uint64_t *out, const uint64_t *a, const uint64_t *b, uint64_t n, int op)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (op < 0 || op > 9) return set_error(ZKGPU_ERR_ARG, "field_selftest: unknown op %d", op);
    if (!n) return 0;
    hipLaunchKernelGGL(k_field_selftest, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, g_ctx.stream, out, a, b, n,
                       op);
    return check_launch("k_field_selftest");
}

int zkgpu_abi_version(void) { return 1; }

const char *zkgpu_last_error(void) { return g_err; }

int zkgpu_init(int device)
{
    Ctx &c = g_ctx;
    if (device < 0) {
        // keep whatever is initialised / current (torch.cuda.set_device in a rank)
        if (c.ready) return 0;
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) cur = 0;
        device = cur;
    }
    if (c.ready && c.device == device) return 0;
    if (c.ready) zkgpu_release();
    int rc;
    if ((rc = check_hip(hipSetDevice(device), "hipSetDevice"))) return rc;
    c.device = device;
    for (int d = 0; d < 2; d++) {
        if ((rc = alloc_dev(&c.rt_small[d], 4096)) || (rc = alloc_dev(&c.tw_lo[d], TW_LEVEL_SIZE)) ||
            (rc = alloc_dev(&c.tw_hi[d], TW_LEVEL_SIZE)))
            return rc;
        uint64_t w12 = h_w(12), w28 = h_w(TW_MAX_LOG);
        if (d) {
            w12 = h_inv(w12);
            w28 = h_inv(w28);
        }
        fill_powers(c.rt_small[d], w12, 1, 1, 4096, c.stream);
        fill_powers(c.tw_lo[d], w28, 1, 1, TW_LEVEL_SIZE, c.stream);
        fill_powers(c.tw_hi[d], w28, TW_LEVEL_SIZE, 1, TW_LEVEL_SIZE, c.stream);
    }
    if ((rc = upload_poseidon_constants(c))) return rc;
    if ((rc = check_launch("init tables"))) return rc;
    if ((rc = check_hip(hipStreamSynchronize(c.stream), "init sync"))) return rc;
    c.ready = true;
    return 0;
}

void zkgpu_release(void)
{
    Ctx &c = g_ctx;
    if (!c.ready) return;
    (void)hipDeviceSynchronize();
    for (int d = 0; d < 2; d++) {
        (void)hipFree(c.rt_small[d]);
        (void)hipFree(c.tw_lo[d]);
        (void)hipFree(c.tw_hi[d]);
    }
    if (c.post_lo) (void)hipFree(c.post_lo);
    if (c.post_hi) (void)hipFree(c.post_hi);
    for (auto &w : c.ws)
        if (w.ptr) (void)hipFree(w.ptr);
    c = Ctx();
}

int zkgpu_set_stream(void *s)
{
    g_ctx.stream = (hipStream_t)s;
    return 0;
}

void *zkgpu_get_stream(void) { return (void *)g_ctx.stream; }

int zkgpu_synchronize(void) { return check_hip(hipStreamSynchronize(g_ctx.stream), "synchronize"); }

// ---------------------------------------------------------------- NTT
int zkgpu_gl_ntt_dev(uint64_t *dst, uint64_t ld_dst, const uint64_t *src, uint64_t ld_src, uint64_t n, uint64_t ncols,
                     int inverse)
{
    int rc;
    if ((rc = require_init())) return rc;
    return ntt_dev(dst, ld_dst, src, ld_src, n, ncols, inverse);
}

uint64_t zkgpu_lde_workspace_bytes(uint64_t n, uint64_t n_ext, uint64_t ncols)
{
    return lde_workspace_bytes(n, n_ext, ncols);
}

void zkgpu_set_lde_batch_cols(uint64_t max_cols) { g_lde_batch_max = max_cols; }

int zkgpu_gl_extend_pol_dev(uint64_t *out, uint64_t ld_out, const uint64_t *in, uint64_t ld_in, uint64_t n_ext,
                            uint64_t n, uint64_t ncols)
{
    int rc;
    if ((rc = require_init())) return rc;
    return extend_pol_dev(out, ld_out, in, ld_in, n_ext, n, ncols);
}

int zkgpu_gl_extend_pol_inplace_dev(uint64_t *base, uint64_t n_ext, uint64_t n, uint64_t ncols)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!ncols || !n) return 0;
    if (!is_pow2(n) || !is_pow2(n_ext) || n_ext < n)
        return set_error(ZKGPU_ERR_ARG, "extend_pol_inplace: sizes must be powers of two with n_ext >= n");
    // batch [c0, c1) reads [c0 n, c1 n) and writes [c0 n_ext, c1 n_ext):
    // the columns below c0, still unread, end at c0 n <= c0 n_ext; within a
    // batch extend_pol_dev stages the whole input (coefficients in workspace
    // 0) before the first output store, on one stream
    const uint64_t batch = lde_batch_cols(n_ext, ncols);
    for (uint64_t c1 = ncols; c1 > 0;) {
        const uint64_t c0 = c1 > batch ? c1 - batch : 0;
        if ((rc = extend_pol_dev(base + c0 * n_ext, n_ext, base + c0 * n, n, n_ext, n, c1 - c0))) return rc;
        c1 = c0;
    }
    return 0;
}

int zkgpu_rows_to_cols_dev(uint64_t *cols, uint64_t ld, const uint64_t *rows, uint64_t nrows, uint64_t ncols)
{
    int rc;
    if ((rc = require_init())) return rc;
    rows_to_cols(rows, cols, nrows, ncols, ld, g_ctx.stream);
    return check_launch("rows_to_cols");
}

int zkgpu_cols_to_rows_dev(uint64_t *rows, const uint64_t *cols, uint64_t ld, uint64_t nrows, uint64_t ncols)
{
    int rc;
    if ((rc = require_init())) return rc;
    cols_to_rows(cols, rows, nrows, ncols, ld, g_ctx.stream);
    return check_launch("cols_to_rows");
}

// host-pointer drop-ins: H2D row-major -> column-major on device -> kernels
// -> row-major -> D2H.  Staging buffers: ws[2] (input cols), ws[3] (output).
int zkgpu_gl_ntt(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t ncols, int inverse)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!n || !ncols) return 0;
    Ctx &c = g_ctx;
    size_t bytes = n * ncols * sizeof(uint64_t);
    uint64_t *rows = workspace(2, bytes);
    uint64_t *cols = workspace(3, bytes);
    if (!rows || !cols) return ZKGPU_ERR_OOM;
    if ((rc = check_hip(hipMemcpyAsync(rows, src, bytes, hipMemcpyHostToDevice, c.stream), "H2D"))) return rc;
    rows_to_cols(rows, cols, n, ncols, n, c.stream);
    if ((rc = ntt_dev(cols, n, cols, n, n, ncols, inverse))) return rc;
    cols_to_rows(cols, rows, n, ncols, n, c.stream);
    if ((rc = check_hip(hipMemcpyAsync(dst, rows, bytes, hipMemcpyDeviceToHost, c.stream), "D2H"))) return rc;
    return check_hip(hipStreamSynchronize(c.stream), "ntt sync");
}

int zkgpu_gl_extend_pol(uint64_t *out, const uint64_t *in, uint64_t n_ext, uint64_t n, uint64_t ncols)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!n || !ncols) return 0;
    if (n_ext < n) return set_error(ZKGPU_ERR_ARG, "extend_pol: n_ext < n");
    Ctx &c = g_ctx;
    size_t in_bytes = n * ncols * sizeof(uint64_t), out_bytes = n_ext * ncols * sizeof(uint64_t);
    uint64_t *rows = workspace(2, out_bytes);
    uint64_t *cols = workspace(3, out_bytes + in_bytes);
    if (!rows || !cols) return ZKGPU_ERR_OOM;
    uint64_t *cin = cols + n_ext * ncols;
    if ((rc = check_hip(hipMemcpyAsync(rows, in, in_bytes, hipMemcpyHostToDevice, c.stream), "H2D"))) return rc;
    rows_to_cols(rows, cin, n, ncols, n, c.stream);
    if ((rc = extend_pol_dev(cols, n_ext, cin, n, n_ext, n, ncols))) return rc;
    cols_to_rows(cols, rows, n_ext, ncols, n_ext, c.stream);
    if ((rc = check_hip(hipMemcpyAsync(out, rows, out_bytes, hipMemcpyDeviceToHost, c.stream), "D2H"))) return rc;
    return check_hip(hipStreamSynchronize(c.stream), "extend_pol sync");
}

// ---------------------------------------------------------------- Poseidon
static int poseidon_one(uint64_t *out, const uint64_t *in, int full)
{
    int rc;
    if ((rc = require_init())) return rc;
    Ctx &c = g_ctx;
    uint64_t *d = workspace(2, 24 * sizeof(uint64_t));
    if (!d) return ZKGPU_ERR_OOM;
    if ((rc = check_hip(hipMemcpyAsync(d, in, 12 * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream), "H2D")))
        return rc;
    if ((rc = poseidon_batch(d + 12, d, 1, full, c.stream))) return rc;
    if ((rc = check_hip(hipMemcpyAsync(out, d + 12, (full ? 12 : 4) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                       c.stream),
                        "D2H")))
        return rc;
    return check_hip(hipStreamSynchronize(c.stream), "poseidon sync");
}

int zkgpu_gl_poseidon_full(uint64_t out[12], const uint64_t in[12]) { return poseidon_one(out, in, 1); }

static uint64_t hp_add(uint64_t a, uint64_t b)  // a, b < p
{
    const uint64_t s = a + b;
    return (s < a || s >= HP) ? s - HP : s;
}
static uint64_t hp_pow7(uint64_t x)
{
    const uint64_t x2 = h_mul(x, x), x3 = h_mul(x2, x), x4 = h_mul(x2, x2);
    return h_mul(x3, x4);
}
// full round r: constants, x^7 on every lane, M[i][j] = MCIRC[(j - i) mod 12] +
// (i == j == 0) * 8 (an MDS row: 13 products of a canonical lane and a
// constant < 2^6, < 2^74, one fold of 2^64)
static void hp_full_round(uint64_t st[12], int r)
{
    static const uint32_t MC[12] = {17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20};
    for (int i = 0; i < 12; i++) st[i] = hp_pow7(hp_add(st[i], ZKGPU_POSEIDON_RC[r * 12 + i]));
    uint64_t t[12];
    for (int i = 0; i < 12; i++) {
        unsigned __int128 acc = (i == 0) ? (unsigned __int128)st[0] * 8 : 0;
        for (int j = 0; j < 12; j++) acc += (unsigned __int128)st[j] * MC[j >= i ? j - i : j + 12 - i];
        const uint64_t lo = (uint64_t)acc, hi = (uint64_t)(acc >> 64);  // hi < 2^10
        const uint64_t hv = (hi << 32) - hi;                            // hi * 2^64 mod p
        uint64_t v = lo + hv;
        if (v < hv) v += 0xFFFFFFFFULL;
        t[i] = v >= HP ? v - HP : v;
    }
    memcpy(st, t, sizeof t);
}

// Host permutation for the transcript (PoseidonGoldilocks::hash_full_result
// on the CPU, transcript.cpp:18-24; the rounds of
// poseidon_g_executor.cpp:201-231): 4 full rounds, the 22 partial rounds in
// the sparse form the device uses (poseidon_gl_sparse.h, perm_sparse in
// csrc/poseidon_perm.hpp: 27 products per round instead of a 12x12 MDS),
// 4 full rounds.  Needs no GPU and no zkgpu_init.
int zkgpu_gl_poseidon_full_host(uint64_t out[12], const uint64_t in[12])
{
    uint64_t st[12];
    for (int i = 0; i < 12; i++) st[i] = in[i] % HP;
    for (int r = 0; r < 4; r++) hp_full_round(st, r);
    {
        uint64_t v[11];
        for (int j = 0; j < 11; j++) v[j] = hp_add(st[1 + j], ZKGPU_PSP_PRE[1 + j]);
        st[0] = hp_add(st[0], ZKGPU_PSP_PRE[0]);
        for (int i = 0; i < 11; i++) {
            uint64_t acc = 0;
            for (int j = 0; j < 11; j++) acc = hp_add(acc, h_mul(v[j], ZKGPU_PSP_D0[i * 11 + j]));
            st[1 + i] = acc;
        }
    }
    for (int k = 0; k < 22; k++) {
        const uint64_t s0 = hp_add(hp_pow7(st[0]), ZKGPU_PSP_POST[k]);
        uint64_t acc = h_mul(s0, 25);
        for (int j = 0; j < 11; j++) acc = hp_add(acc, h_mul(st[1 + j], ZKGPU_PSP_W[k * 11 + j]));
        for (int j = 0; j < 11; j++) st[1 + j] = hp_add(st[1 + j], h_mul(s0, ZKGPU_PSP_V[k * 11 + j]));
        st[0] = acc;
    }
    for (int r = 26; r < 30; r++) hp_full_round(st, r);
    memcpy(out, st, sizeof st);
    return 0;
}
int zkgpu_gl_poseidon_hash(uint64_t out[4], const uint64_t in[12]) { return poseidon_one(out, in, 0); }

int zkgpu_gl_poseidon_batch_dev(uint64_t *out, const uint64_t *in, uint64_t n, int full)
{
    int rc;
    if ((rc = require_init())) return rc;
    return poseidon_batch(out, in, n, full, g_ctx.stream);
}

int zkgpu_gl_linear_hash(uint64_t out[4], const uint64_t *in, uint64_t size)
{
    int rc;
    if ((rc = require_init())) return rc;
    Ctx &c = g_ctx;
    uint64_t *d = workspace(2, (size + 4) * sizeof(uint64_t));
    if (!d) return ZKGPU_ERR_OOM;
    if (size && (rc = check_hip(hipMemcpyAsync(d + 4, in, size * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream),
                                "H2D")))
        return rc;
    // one row of `size` columns, column-major with ld = 1
    if ((rc = merkle_leaves_cols(d, d + 4, size, 1, 1, c.stream))) return rc;
    if ((rc = check_hip(hipMemcpyAsync(out, d, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream), "D2H")))
        return rc;
    return check_hip(hipStreamSynchronize(c.stream), "linear_hash sync");
}

// ---------------------------------------------------------------- Merkle
uint64_t zkgpu_gl_merkle_num_elements(uint64_t nrows) { return nrows ? 4 * nrows + 4 * (nrows - 1) : 0; }

int zkgpu_gl_merkletree_dev(uint64_t *nodes, const uint64_t *src, uint64_t ld, uint64_t ncols, uint64_t nrows)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!nrows) return 0;
    if (!is_pow2(nrows)) return set_error(ZKGPU_ERR_ARG, "merkletree: nrows must be a power of two");
    if ((rc = merkle_leaves_cols(nodes, src, ncols, nrows, ld, g_ctx.stream))) return rc;
    return merkle_levels(nodes, nrows, g_ctx.stream);
}

int zkgpu_gl_merkletree2_dev(uint64_t *nodes, const uint64_t *src, const uint64_t *src2, uint64_t ld, uint64_t split,
                             uint64_t ncols, uint64_t nrows)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!nrows) return 0;
    if (!is_pow2(nrows)) return set_error(ZKGPU_ERR_ARG, "merkletree2: nrows must be a power of two");
    if (split > ncols || (split < ncols && split % 8))
        return set_error(ZKGPU_ERR_ARG, "merkletree2: split %llu must be a multiple of 8 up to ncols",
                         (unsigned long long)split);
    if ((rc = merkle_leaves_cols(nodes, src, ncols, nrows, ld, g_ctx.stream, src2, split))) return rc;
    return merkle_levels(nodes, nrows, g_ctx.stream);
}

int zkgpu_gl_merkletree_rows_dev(uint64_t *nodes, const uint64_t *src, uint64_t ncols, uint64_t nrows)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!nrows) return 0;
    if (!is_pow2(nrows)) return set_error(ZKGPU_ERR_ARG, "merkletree: nrows must be a power of two");
    if ((rc = merkle_leaves_rows(nodes, src, ncols, nrows, g_ctx.stream))) return rc;
    return merkle_levels(nodes, nrows, g_ctx.stream);
}

int zkgpu_gl_merkletree(uint64_t *nodes, const uint64_t *src, uint64_t ncols, uint64_t nrows)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!nrows) return 0;
    if (!is_pow2(nrows)) return set_error(ZKGPU_ERR_ARG, "merkletree: nrows must be a power of two");
    Ctx &c = g_ctx;
    size_t src_bytes = nrows * ncols * sizeof(uint64_t);
    size_t nodes_bytes = zkgpu_gl_merkle_num_elements(nrows) * sizeof(uint64_t);
    uint64_t *rows = workspace(2, src_bytes + 8);
    uint64_t *dn = workspace(3, nodes_bytes + src_bytes + 8);
    if (!rows || !dn) return ZKGPU_ERR_OOM;
    uint64_t *cols = dn + zkgpu_gl_merkle_num_elements(nrows);
    if (src_bytes &&
        (rc = check_hip(hipMemcpyAsync(rows, src, src_bytes, hipMemcpyHostToDevice, c.stream), "H2D")))
        return rc;
    rows_to_cols(rows, cols, nrows, ncols, nrows, c.stream);
    if ((rc = merkle_leaves_cols(dn, cols, ncols, nrows, nrows, c.stream))) return rc;
    if ((rc = merkle_levels(dn, nrows, c.stream))) return rc;
    if ((rc = check_hip(hipMemcpyAsync(nodes, dn, nodes_bytes, hipMemcpyDeviceToHost, c.stream), "D2H"))) return rc;
    return check_hip(hipStreamSynchronize(c.stream), "merkletree sync");
}

int zkgpu_gl_merkle_open_dev(uint64_t *vals_out, uint64_t *sibs_out, const uint64_t *nodes, const uint64_t *src,
                             uint64_t ld, uint64_t ncols, uint64_t nrows, const uint64_t *idx, uint64_t nq)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!nq) return 0;
    Ctx &c = g_ctx;
    uint32_t nlev = log2u(nrows);
    for (uint64_t q = 0; q < nq; q++)
        if (idx[q] >= nrows) return set_error(ZKGPU_ERR_ARG, "merkle_open: index %llu >= nrows", (unsigned long long)idx[q]);
    size_t nv = nq * ncols, ns = nq * nlev * 4;
    uint64_t *d = workspace(2, (nq + nv + ns + 1) * sizeof(uint64_t));
    if (!d) return ZKGPU_ERR_OOM;
    uint64_t *didx = d, *dv = d + nq, *ds = d + nq + nv;
    if ((rc = check_hip(hipMemcpyAsync(didx, idx, nq * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream), "H2D")))
        return rc;
    if ((rc = merkle_open_cols(dv, ds, nodes, src, ncols, nrows, ld, didx, nq, c.stream))) return rc;
    if (nv && (rc = check_hip(hipMemcpyAsync(vals_out, dv, nv * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream),
                              "D2H")))
        return rc;
    if (ns && (rc = check_hip(hipMemcpyAsync(sibs_out, ds, ns * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream),
                              "D2H")))
        return rc;
    return check_hip(hipStreamSynchronize(c.stream), "merkle_open sync");
}

// ---------------------------------------------------------------- const tree
uint64_t zkgpu_const_tree_num_elements(uint64_t n_pols, uint32_t n_bits_ext)
{
    const uint64_t n_ext = 1ULL << n_bits_ext;
    return 2 + n_pols * n_ext + zkgpu_gl_merkle_num_elements(n_ext);
}

int zkgpu_build_const_tree(uint64_t *tree_out, const uint64_t *const_pols, uint64_t n_pols, uint32_t n_bits,
                           uint32_t n_bits_ext)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (n_bits_ext < n_bits || n_bits_ext > TW_MAX_LOG)
        return set_error(ZKGPU_ERR_ARG, "const_tree: bad nBits %u / nBitsExt %u", n_bits, n_bits_ext);
    Ctx &c = g_ctx;
    const uint64_t n = 1ULL << n_bits, n_ext = 1ULL << n_bits_ext;
    const uint64_t n_nodes = zkgpu_gl_merkle_num_elements(n_ext);
    tree_out[0] = n_pols;  // Goldilocks::fromU64(nPols), fromU64(nExt)
    tree_out[1] = n_ext;
    const size_t in_bytes = n * n_pols * sizeof(uint64_t), out_bytes = n_ext * n_pols * sizeof(uint64_t);
    uint64_t *rows = workspace(2, out_bytes + 8);
    uint64_t *cols = workspace(3, out_bytes + in_bytes + n_nodes * sizeof(uint64_t) + 8);
    if (!rows || !cols) return ZKGPU_ERR_OOM;
    uint64_t *cin = cols + n_ext * n_pols;
    uint64_t *nodes = cin + n * n_pols;
    if (n_pols) {
        if ((rc = check_hip(hipMemcpyAsync(rows, const_pols, in_bytes, hipMemcpyHostToDevice, c.stream), "H2D")))
            return rc;
        rows_to_cols(rows, cin, n, n_pols, n, c.stream);
        if ((rc = extend_pol_dev(cols, n_ext, cin, n, n_ext, n, n_pols))) return rc;  // interpolate()
    }
    if ((rc = merkle_leaves_cols(nodes, cols, n_pols, n_ext, n_ext, c.stream))) return rc;
    if ((rc = merkle_levels(nodes, n_ext, c.stream))) return rc;
    if (n_pols) {
        cols_to_rows(cols, rows, n_ext, n_pols, n_ext, c.stream);
        if ((rc = check_hip(hipMemcpyAsync(tree_out + 2, rows, out_bytes, hipMemcpyDeviceToHost, c.stream), "D2H")))
            return rc;
    }
    if ((rc = check_hip(hipMemcpyAsync(tree_out + 2 + n_ext * n_pols, nodes, n_nodes * sizeof(uint64_t),
                                       hipMemcpyDeviceToHost, c.stream),
                        "D2H")))
        return rc;
    return check_hip(hipStreamSynchronize(c.stream), "const_tree sync");
}

// ---------------------------------------------------------------- executor hand-off
// block loop of the loaders: block b's H2D copy into stage half b & 1 on a copy
// stream, its transpose into the columns on stream ts once copied; a half is
// refilled only after its transpose has read it.  Returns with the work queued
// (ts, the copy stream), not finished.
static int load_rows_blocks(uint64_t *cols, uint64_t ld, const uint64_t *rows, uint64_t nrows, uint64_t ncols,
                            uint64_t block_rows, uint64_t *stage, hipStream_t cs, hipStream_t ts, hipEvent_t copied[2],
                            hipEvent_t freed[2])
{
    int rc = 0;
    const uint64_t nblocks = (nrows + block_rows - 1) / block_rows;
    for (uint64_t b = 0; b < nblocks && !rc; b++) {
        const int k = (int)(b & 1);
        const uint64_t r0 = b * block_rows, nr = std::min(block_rows, nrows - r0);
        uint64_t *buf = stage + (size_t)k * block_rows * ncols;
        if (b >= 2 && (rc = check_hip(hipStreamWaitEvent(cs, freed[k], 0), "wait"))) break;
        if ((rc = check_hip(hipMemcpyAsync(buf, rows + r0 * ncols, nr * ncols * sizeof(uint64_t),
                                           hipMemcpyHostToDevice, cs),
                            "H2D")))
            break;
        if ((rc = check_hip(hipEventRecord(copied[k], cs), "record"))) break;
        if ((rc = check_hip(hipStreamWaitEvent(ts, copied[k], 0), "wait"))) break;
        rows_to_cols(buf, cols + r0, nr, ncols, ld, ts);
        if ((rc = check_hip(hipEventRecord(freed[k], ts), "record"))) break;
    }
    return rc;
}

static uint64_t load_block_rows(uint64_t block_rows, uint64_t nrows, uint64_t ncols)
{
    if (!block_rows) block_rows = std::max<uint64_t>(1, (64ULL << 20) / (ncols * sizeof(uint64_t)));  // ~64 MB
    return std::min(block_rows, nrows);
}

// one load on its own streams (transposes on ts): the shared body of the
// synchronous and the background loader
// `after` (optional): an event both streams wait for before their first
// command -- the background loader's streams are non-blocking and would
// otherwise overtake work the caller queued on the library stream into the
// same buffers (the zeroing memsets of freshly allocated cols / stage).
static int load_rows_streams(uint64_t *cols, uint64_t ld, const uint64_t *rows, uint64_t nrows, uint64_t ncols,
                             uint64_t block_rows, uint64_t *stage, hipStream_t ts, bool register_host,
                             hipEvent_t after = nullptr)
{
    int rc = 0;
    const size_t total = nrows * ncols * sizeof(uint64_t);
    bool registered = false;
    if (register_host) {
        if ((rc = check_hip(hipHostRegister((void *)rows, total, hipHostRegisterDefault), "hipHostRegister")))
            return rc;
        registered = true;
    }
    hipStream_t cs = nullptr;
    hipEvent_t copied[2] = {nullptr, nullptr}, freed[2] = {nullptr, nullptr};
    rc = check_hip(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "copy stream");
    for (int k = 0; k < 2 && !rc; k++) {
        rc = check_hip(hipEventCreateWithFlags(&copied[k], hipEventDisableTiming), "event");
        if (!rc) rc = check_hip(hipEventCreateWithFlags(&freed[k], hipEventDisableTiming), "event");
    }
    if (!rc && after) rc = check_hip(hipStreamWaitEvent(cs, after, 0), "wait");
    if (!rc && after) rc = check_hip(hipStreamWaitEvent(ts, after, 0), "wait");
    if (!rc) rc = load_rows_blocks(cols, ld, rows, nrows, ncols, block_rows, stage, cs, ts, copied, freed);
    if (!rc) rc = check_hip(hipStreamSynchronize(ts), "load_rows sync");
    if (cs) (void)hipStreamSynchronize(cs);
    for (int k = 0; k < 2; k++) {
        if (copied[k]) (void)hipEventDestroy(copied[k]);
        if (freed[k]) (void)hipEventDestroy(freed[k]);
    }
    if (cs) (void)hipStreamDestroy(cs);
    if (registered) (void)hipHostUnregister((void *)rows);
    return rc ? rc : check_launch("rows_to_cols");
}

int zkgpu_load_rows_dev(uint64_t *cols, uint64_t ld, const uint64_t *rows, uint64_t nrows, uint64_t ncols,
                        uint64_t block_rows, int register_host)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!nrows || !ncols) return 0;
    if (ld < nrows) return set_error(ZKGPU_ERR_ARG, "load_rows: ld %llu < nrows", (unsigned long long)ld);
    block_rows = load_block_rows(block_rows, nrows, ncols);
    uint64_t *stage = workspace(2, 2 * block_rows * ncols * sizeof(uint64_t));
    if (!stage) return ZKGPU_ERR_OOM;
    return load_rows_streams(cols, ld, rows, nrows, ncols, block_rows, stage, g_ctx.stream, register_host != 0);
}

// Background loader (zkgpu_load_rows_async): the same block loop in a host
// thread of its own, on streams of its own, so a proof's kernels on the
// library stream run while the next trace crosses PCIe.  A pageable source
// is staged through the driver by the calling thread of the copy, which is
// why the copies need a thread and not only a stream.
struct LoadTicket {
    std::thread th;
    int rc = 0;
    hipEvent_t after = nullptr;  // the library stream's work queued before the load
    char err[512] = "";          // the loader thread's error text (g_err is thread-local)
};

uint64_t zkgpu_load_rows_stage_bytes(uint64_t nrows, uint64_t ncols, uint64_t block_rows)
{
    if (!nrows || !ncols) return 0;
    return 2 * load_block_rows(block_rows, nrows, ncols) * ncols * sizeof(uint64_t);
}

int zkgpu_load_rows_async(uint64_t *cols, uint64_t ld, const uint64_t *rows, uint64_t nrows, uint64_t ncols,
                          uint64_t block_rows, uint64_t *stage, uint64_t stage_bytes, void **ticket)
{
    int rc;
    *ticket = nullptr;
    if ((rc = require_init())) return rc;
    if (ld < nrows) return set_error(ZKGPU_ERR_ARG, "load_rows_async: ld %llu < nrows", (unsigned long long)ld);
    block_rows = load_block_rows(block_rows, nrows, ncols);
    if (nrows && ncols && (!stage || stage_bytes < 2 * block_rows * ncols * sizeof(uint64_t)))
        return set_error(ZKGPU_ERR_ARG, "load_rows_async: stage of %llu bytes < 2 blocks (%llu)",
                         (unsigned long long)stage_bytes, (unsigned long long)(2 * block_rows * ncols * 8));
    LoadTicket *t = new (std::nothrow) LoadTicket();
    if (!t) return set_error(ZKGPU_ERR_OOM, "load_rows_async: ticket");
    if (nrows && ncols) {
        if ((rc = check_hip(hipEventCreateWithFlags(&t->after, hipEventDisableTiming), "event")) ||
            (rc = check_hip(hipEventRecord(t->after, g_ctx.stream), "record"))) {
            if (t->after) (void)hipEventDestroy(t->after);
            delete t;
            return rc;
        }
    }
    const int device = g_ctx.device;
    try {
        t->th = std::thread([=] {
        if (!nrows || !ncols) return;
        int r = check_hip(hipSetDevice(device), "hipSetDevice (loader)");
        hipStream_t ts = nullptr;
        if (!r) r = check_hip(hipStreamCreateWithFlags(&ts, hipStreamNonBlocking), "loader stream");
        if (!r) r = load_rows_streams(cols, ld, rows, nrows, ncols, block_rows, stage, ts, false, t->after);
        if (ts) (void)hipStreamDestroy(ts);
        if (r) snprintf(t->err, sizeof t->err, "%s", g_err);
        t->rc = r;
        });
    } catch (...) {  // no thread: nothing started
        if (t->after) (void)hipEventDestroy(t->after);
        delete t;
        return set_error(ZKGPU_ERR_ARG, "load_rows_async: cannot start the loader thread");
    }
    *ticket = t;
    return 0;
}

int zkgpu_load_wait(void *ticket)
{
    if (!ticket) return 0;
    LoadTicket *t = (LoadTicket *)ticket;
    if (t->th.joinable()) t->th.join();
    const int rc = t->rc;
    if (rc) set_error(rc, "%s", t->err);  // the loader's message, on the waiting thread
    if (t->after) (void)hipEventDestroy(t->after);
    delete t;
    return rc;
}

// ---------------------------------------------------------------- device memory
int zkgpu_dev_malloc(void **ptr, uint64_t bytes)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (hipMalloc(ptr, bytes ? bytes : 8) != hipSuccess) {
        *ptr = nullptr;
        return set_error(ZKGPU_ERR_OOM, "hipMalloc(%llu) failed", (unsigned long long)bytes);
    }
    return 0;
}
int zkgpu_dev_free(void *ptr) { return ptr ? check_hip(hipFree(ptr), "hipFree") : 0; }
int zkgpu_memcpy_h2d(void *dst, const void *src, uint64_t bytes)
{
    if (!bytes) return 0;
    int rc = check_hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, g_ctx.stream), "H2D");
    return rc ? rc : check_hip(hipStreamSynchronize(g_ctx.stream), "H2D sync");
}
int zkgpu_memcpy_d2h(void *dst, const void *src, uint64_t bytes)
{
    if (!bytes) return 0;
    int rc = check_hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, g_ctx.stream), "D2H");
    return rc ? rc : check_hip(hipStreamSynchronize(g_ctx.stream), "D2H sync");
}
int zkgpu_memcpy_d2d(void *dst, const void *src, uint64_t bytes)
{
    if (!bytes) return 0;
    return check_hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, g_ctx.stream), "D2D");
}
int zkgpu_memset_dev(void *dst, int value, uint64_t bytes)
{
    if (!bytes) return 0;
    return check_hip(hipMemsetAsync(dst, value, bytes, g_ctx.stream), "memset");
}

// ---------------------------------------------------------------- STARK stages
// small host arrays staged through a grow-only device buffer (ws slot 3 is the
// host-API staging area; stage params use their own allocation)
static uint64_t *g_param = nullptr;
static size_t g_param_bytes = 0;
static char *param_buf(size_t bytes)
{
    if (bytes > g_param_bytes) {
        (void)hipStreamSynchronize(g_ctx.stream);
        if (g_param) (void)hipFree(g_param);
        g_param = nullptr;
        if (hipMalloc((void **)&g_param, bytes) != hipSuccess) {
            g_param_bytes = 0;
            return nullptr;
        }
        g_param_bytes = bytes;
    }
    return (char *)g_param;
}

int zkgpu_rand_cols_dev(uint64_t *base, uint64_t ld, const uint32_t *cols, uint32_t ncols, uint64_t nrows,
                        uint64_t seed, uint64_t stream)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!ncols) return 0;
    char *p = param_buf(ncols * 4);
    if (!p) return set_error(ZKGPU_ERR_OOM, "param buffer");
    if ((rc = check_hip(hipMemcpyAsync(p, cols, ncols * 4, hipMemcpyHostToDevice, g_ctx.stream), "H2D"))) return rc;
    if ((rc = check_hip(hipStreamSynchronize(g_ctx.stream), "rand_cols param upload"))) return rc;
    return rand_cols(base, ld, (const uint32_t *)p, ncols, nrows, seed, stream, 0, ~0ULL, g_ctx.stream);
}

int zkgpu_rand_cols_rows_dev(uint64_t *base, uint64_t ld, const uint32_t *cols, uint32_t ncols, uint64_t row0,
                             uint64_t nrows, uint32_t log_n, uint64_t seed, uint64_t stream)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!ncols || !nrows) return 0;
    if (log_n > 40 || ncols > 65535 || nrows > ld) return set_error(ZKGPU_ERR_ARG, "rand_cols_rows: bad shape");
    char *p = param_buf(ncols * 4);
    if (!p) return set_error(ZKGPU_ERR_OOM, "param buffer");
    if ((rc = check_hip(hipMemcpyAsync(p, cols, ncols * 4, hipMemcpyHostToDevice, g_ctx.stream), "H2D"))) return rc;
    if ((rc = check_hip(hipStreamSynchronize(g_ctx.stream), "rand_cols param upload"))) return rc;
    return rand_cols(base, ld, (const uint32_t *)p, ncols, nrows, seed, stream, row0, (1ULL << log_n) - 1,
                     g_ctx.stream);
}

int zkgpu_copy_rows_dev(uint64_t *dst, uint64_t dst_ld, uint64_t dst_row0, const uint32_t *dst_cols,
                        const uint64_t *src, uint64_t src_ld, uint64_t src_row0, uint32_t src_log_mod,
                        const uint32_t *src_cols, uint32_t ncols, uint64_t nrows)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!ncols || !nrows) return 0;
    if (!dst || !src || ncols > 65535 || src_log_mod > 63 || dst_row0 + nrows > dst_ld ||
        (!src_log_mod && src_row0 + nrows > src_ld) || (src_log_mod && (1ULL << src_log_mod) > src_ld))
        return set_error(ZKGPU_ERR_ARG, "copy_rows: rows outside the buffers' leading dimensions");
    const size_t nd = dst_cols ? ncols : 0, ns = src_cols ? ncols : 0;
    char *p = param_buf((nd + ns) * 4 + 8);
    if (!p) return set_error(ZKGPU_ERR_OOM, "param buffer");
    if (nd && (rc = check_hip(hipMemcpyAsync(p, dst_cols, nd * 4, hipMemcpyHostToDevice, g_ctx.stream), "H2D")))
        return rc;
    if (ns && (rc = check_hip(hipMemcpyAsync(p + nd * 4, src_cols, ns * 4, hipMemcpyHostToDevice, g_ctx.stream), "H2D")))
        return rc;
    if ((nd || ns) && (rc = check_hip(hipStreamSynchronize(g_ctx.stream), "copy_rows param upload"))) return rc;
    return copy_rows(dst, dst_ld, dst_row0, nd ? (const uint32_t *)p : nullptr, src, src_ld, src_row0,
                     src_log_mod ? (1ULL << src_log_mod) - 1 : ~0ULL, ns ? (const uint32_t *)(p + nd * 4) : nullptr,
                     ncols, nrows, g_ctx.stream);
}

int zkgpu_device_memory(uint64_t *free_bytes, uint64_t *total_bytes)
{
    int rc;
    if ((rc = require_init())) return rc;
    size_t f = 0, t = 0;
    if ((rc = check_hip(hipMemGetInfo(&f, &t), "hipMemGetInfo"))) return rc;
    if (free_bytes) *free_bytes = f;
    if (total_bytes) *total_bytes = t;
    return 0;
}

static inline uint64_t h_add(uint64_t a, uint64_t b)
{
    const uint64_t s = a + b;  // a, b < p
    return (s < a || s >= HP) ? s - HP : s;
}

// Temp-slot allocation for a ZXP program.  Program producers (the synthetic
// builder, a chelpers converter) may give every intermediate its own temp;
// the LDS footprint per workgroup is (slots x 64 rows x 8 B), which bounds
// occupancy.  Each temp identity lives over [first occurrence, last
// occurrence]; a linear scan packs the intervals of each pool (base / ext)
// into the fewest slots.  An interval may start at the instruction where
// another ends: the interpreter loads both sources before it stores the
// destination.  The operand table is rewritten (duplicates are harmless).
static void zxp_alloc_slots(const zxp_instr *in, uint32_t n_instr, std::vector<zxp_operand> &op, uint32_t &n_tmp1,
                            uint32_t &n_tmp3)
{
    for (int pool = 0; pool < 2; pool++) {
        const uint32_t kind = pool ? ZXP_TMP3 : ZXP_TMP1;
        const uint32_t n_id = pool ? n_tmp3 : n_tmp1;
        std::vector<uint32_t> first(n_id, UINT32_MAX), last(n_id, 0);
        for (uint32_t k = 0; k < n_instr; k++) {
            const uint32_t refs[3] = {in[k].dst, in[k].a, in[k].op == ZXP_COPY ? in[k].a : in[k].b};
            for (uint32_t r : refs)
                if (op[r].kind == kind) {
                    const uint32_t id = op[r].a;
                    first[id] = std::min(first[id], k);
                    last[id] = std::max(last[id], k);
                }
        }
        std::vector<uint32_t> order;
        for (uint32_t id = 0; id < n_id; id++)
            if (first[id] != UINT32_MAX) order.push_back(id);
        std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return first[x] < first[y]; });
        std::vector<uint32_t> slot_of(n_id, 0), slot_end;
        for (uint32_t id : order) {
            uint32_t s = 0;
            while (s < slot_end.size() && slot_end[s] > first[id]) s++;
            if (s == slot_end.size()) slot_end.push_back(0);
            slot_end[s] = last[id];
            slot_of[id] = s;
        }
        for (auto &o : op)
            if (o.kind == kind) o.a = slot_of[o.a];
        const uint32_t used = (uint32_t)std::max<size_t>(slot_end.size(), 1);
        (pool ? n_tmp3 : n_tmp1) = used;
    }
}

// log_dom: rows evaluated (2^log_dom); log_omega: x_i = x_start * w_{2^log_omega}^i and zhInv's N =
// 2^(log_omega - extend_bits); wrap: shifted reads wrap mod 2^log_dom, else halo rows follow the block
// zhInv tables (<= 64 words) on the device, one per (log omega, extend
// bits), uploaded once: the compiled expression kernels read them and need
// no per-call upload (and no stream sync for a pageable source)
// (keyed by device too: zkgpu_init may switch devices)
static const uint64_t *zh_table(uint32_t log_omega, uint32_t eb, const uint64_t *zhv, size_t n)
{
    static std::mutex mu;
    static std::map<std::pair<int, std::pair<uint32_t, uint32_t>>, uint64_t *> tabs;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(g_ctx.device, std::make_pair(log_omega, eb));
    auto it = tabs.find(key);
    if (it != tabs.end()) return it->second;
    uint64_t *d = nullptr;
    if (check_hip(hipMalloc((void **)&d, 64 * 8), "zxp: zhInv table")) return nullptr;
    if (check_hip(hipMemcpy(d, zhv, n * 8, hipMemcpyHostToDevice), "zxp: zhInv table")) {
        (void)hipFree(d);
        return nullptr;
    }
    tabs[key] = d;
    return d;
}

static int zxp_eval_impl(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd, uint32_t n_tmp1,
                         uint32_t n_tmp3, const zkgpu_sections *sections, uint32_t log_dom, uint32_t log_omega,
                         int wrap, const uint64_t *challenges, const uint64_t *publics, uint32_t n_publics,
                         const uint64_t *evals, uint32_t n_evals, const uint64_t *xdiv, const uint64_t *xdivw,
                         uint32_t extend_bits, uint64_t x_start, int force_interp = 0)
{
    int rc;
    if ((rc = require_init())) return rc;
    const uint32_t n_instr0 = n_instr, n_tmp1_0 = n_tmp1, n_tmp3_0 = n_tmp3;
    const void *opnd0 = opnd;
    if (log_omega > TW_MAX_LOG || log_dom > log_omega) return set_error(ZKGPU_ERR_ARG, "zxp: domain too large");
    if (extend_bits > log_omega) return set_error(ZKGPU_ERR_ARG, "zxp: extend bits exceed the domain");
    // validate operands on the host (no out-of-range reads in the kernel)
    const zxp_instr *in = (const zxp_instr *)instr;
    const zxp_operand *op = (const zxp_operand *)opnd;
    for (uint32_t k = 0; k < n_instr; k++)
        if (in[k].dst >= n_opnd || in[k].a >= n_opnd || (in[k].op != ZXP_COPY && in[k].b >= n_opnd) || in[k].op > 3)
            return set_error(ZKGPU_ERR_ARG, "zxp: instruction %u out of range", k);
    for (uint32_t k = 0; k < n_opnd; k++) {
        const zxp_operand &o = op[k];
        bool bad = false;
        switch (o.kind) {
        case ZXP_TMP1: bad = o.a >= n_tmp1; break;
        case ZXP_TMP3: bad = o.a >= n_tmp3; break;
        case ZXP_COL:
        case ZXP_COL3: {
            const uint32_t w = o.kind == ZXP_COL3 ? 3 : 1;
            const int32_t sh = (int32_t)o.c;
            // without wrap-around a shifted read touches halo rows [2^log_dom, 2^log_dom + sh)
            const uint64_t need = (1ULL << log_dom) + (wrap ? 0 : (uint64_t)(sh > 0 ? sh : 0));
            bad = o.a >= SEC_COUNT || !sections->sec[o.a] || (uint64_t)o.b + w > sections->ncols[o.a] ||
                  sections->ld[o.a] < need || (!wrap && sh < 0);
            break;
        }
        case ZXP_CHAL: bad = o.a >= 8; break;
        case ZXP_PUB: bad = o.a >= n_publics; break;
        case ZXP_EVAL: bad = o.a >= n_evals; break;
        case ZXP_XDIV: bad = !xdiv; break;
        case ZXP_XDIVW: bad = !xdivw; break;
        case ZXP_LIT:
        case ZXP_X:
        case ZXP_ZI: break;
        default: bad = true;
        }
        if (bad) return set_error(ZKGPU_ERR_ARG, "zxp: operand %u (kind %u) invalid", k, o.kind);
    }
    // compile (csrc/zxp_compile.cpp): linear-combination fusion + SSA slots.
    // ZKGPU_ZXP_FUSE=0 runs the source program as is (slot packing only).
    const char *env_fuse = getenv("ZKGPU_ZXP_FUSE");
    const char *env_terms = getenv("ZKGPU_ZXP_MAX_TERMS");
    const int fuse = env_fuse ? atoi(env_fuse) : 1;
    const uint32_t max_terms = env_terms ? (uint32_t)atoi(env_terms) : 0u;
    // The compiled program runs as a run-time compiled straight-line kernel
    // (csrc/zxp_jit.hip, compiled once per program per process) on domains of
    // 2^16 rows and more, where it pays for its ~1-2 s compile; smaller
    // domains use the interpreter.  ZKGPU_ZXP_JIT=0 never, =2 always.
    const char *env_jit = getenv("ZKGPU_ZXP_JIT");
    const int jit_mode = env_jit ? atoi(env_jit) : 1;
    // (the compiled kernels address a column with a 32-bit byte offset:
    // domains up to 2^28 rows plus their halo)
    const bool use_jit = !force_interp && fuse && log_dom <= 28 && (jit_mode == 2 || (jit_mode == 1 && log_dom >= 16));
    std::vector<zxp_operand> opv;
    const zxp_instr *pin = in;
    const zxp_term *terms = nullptr;
    const uint64_t *csts = nullptr;
    uint32_t n_terms = 0;
    if (fuse) {
        zxp_compiled cp;
        // (one compile serves both paths: measured, longer DOTs / fused DOT
        // column passes / no live-temporary cap made the compiled kernels slower)
        if ((rc = zkgpu_zxp_compile(instr, n_instr, opnd, n_opnd, n_tmp1, n_tmp3, challenges, publics, n_publics,
                                    evals, n_evals, max_terms, &cp)))
            return rc;
        pin = cp.instr;
        n_instr = cp.n_instr;
        opv.assign(cp.opnd, cp.opnd + cp.n_opnd);
        terms = cp.term;
        n_terms = cp.n_term;
        csts = cp.cst;
        n_tmp1 = cp.n_tmp1;
        n_tmp3 = cp.n_tmp3;
    } else {
        opv.assign(op, op + n_opnd);
        zxp_alloc_slots(in, n_instr, opv, n_tmp1, n_tmp3);
    }
    const uint32_t n_dot_terms = [&] {
        uint32_t c = 0;
        for (uint32_t t = 0; t < n_terms; t++) c += terms[t].src != ZXP_TERM_ONE;
        return c;
    }();
    const uint32_t n_logz = extend_bits;
    const size_t zh = (size_t)1 << n_logz;
    if (zh > 64) return set_error(ZKGPU_ERR_ARG, "zxp: extend bits > 6");
    // zhInv[j] = 1/(7^N * W[eb]^j - 1)  (zhInv.cpp:7-31), N = 2^(log_dom - eb)
    uint64_t zhv[64];
    {
        uint64_t sn = h_pow(7, 1ULL << (log_omega - extend_bits));
        uint64_t we = h_w(extend_bits), w = 1;
        for (size_t j = 0; j < zh; j++) {
            const uint64_t x = h_mul(sn, w);  // < HP
            zhv[j] = h_inv(x ? x - 1 : HP - 1);
            w = h_mul(w, we);
        }
    }
    for (uint32_t k = 0; k < n_opnd; k++)
        if ((op[k].kind == ZXP_COL || op[k].kind == ZXP_COL3) && sections->ld[op[k].a] > 0xFFFFFFFFULL)
            return set_error(ZKGPU_ERR_ARG, "zxp: section %u stride exceeds 2^32", op[k].a);
    hipStream_t s = g_ctx.stream;
    // algorithmic bytes: every distinct column operand read once per row + written columns
    double alg_bytes = 0;
    for (uint32_t k = 0; k < n_opnd; k++) {
        const uint32_t kind = op[k].kind;
        alg_bytes += kind == ZXP_COL ? 1 : (kind == ZXP_COL3 || kind == ZXP_XDIV || kind == ZXP_XDIVW) ? 3 : 0;
    }
    alg_bytes *= 8.0 * (double)(1ULL << log_dom);
    if (use_jit) {
        // the compiled kernels take their own tables (csrc/zxp_jit.hip): no
        // interpreter records, no upload or stream sync here, so the host
        // prepares them while earlier work still runs on the stream
        for (uint32_t k = 0; k < n_instr; k++) {
            const zxp_instr &I = pin[k];
            if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
                for (uint32_t t = I.a; t < I.a + I.b; t++) {
                    if (terms[t].src == ZXP_TERM_ONE) continue;
                    const uint32_t kind = opv[terms[t].src].kind;
                    if (kind != ZXP_COL && kind != ZXP_TMP1 && kind != ZXP_TMP3)
                        return set_error(ZKGPU_ERR_ARG, "zxp: DOT term source kind %u", kind);
                }
            }
            const uint32_t dk = opv[I.dst].kind;
            if (dk != ZXP_TMP1 && dk != ZXP_TMP3 && dk != ZXP_COL && dk != ZXP_COL3)
                return set_error(ZKGPU_ERR_ARG, "zxp: instruction %u writes a read-only operand", k);
        }
        const uint64_t *zh_dev = zh_table(log_omega, extend_bits, zhv, zh);
        if (!zh_dev) return -1;
        ZxpJitIn J;
        J.ins = pin;
        J.n_instr = n_instr;
        J.opnd = opv.data();
        J.n_opnd = (uint32_t)opv.size();
        J.terms = terms;
        J.csts = csts;
        J.n_tmp1 = n_tmp1;
        J.n_tmp3 = n_tmp3;
        J.sections = sections;
        J.log_dom = log_dom;
        J.log_omega = log_omega;
        J.wrap = wrap ? 1u : 0u;
        J.challenges = challenges;
        J.publics = publics;
        J.evals = evals;
        J.xdiv = xdiv;
        J.xdivw = xdivw;
        J.zh_dev = zh_dev;
        J.zmask = (uint32_t)(zh - 1);
        J.x_start = x_start % HP;
        J.bytes = alg_bytes;
        J.dot_loop_min = 8;  // (zxp_jit.hip zkgpu_zxp_jit_source uses the same settings)
        J.waves_per_eu = 0;
        J.force_split = 0;
        J.scratch = nullptr;
        J.scratch_ld = 0;
        rc = zxp_jit_run(J, s);
        if (rc <= 0) return rc;  // launched, or an error
        // 1 = shape unsupported: compile for the interpreter instead
        return zxp_eval_impl(instr, n_instr0, opnd0, n_opnd, n_tmp1_0, n_tmp3_0, sections, log_dom, log_omega, wrap,
                             challenges, publics, n_publics, evals, n_evals, xdiv, xdivw, extend_bits, x_start, 1);
    }
    size_t off_prog = 0;
    size_t off_terms = off_prog + (size_t)std::max<uint32_t>(n_instr, 1) * sizeof(ZOp);
    size_t off_zh = off_terms + (size_t)n_dot_terms * sizeof(ZTerm);
    size_t total = off_zh + zh * 8 + 16;
    char *p = param_buf(total);
    if (!p) return set_error(ZKGPU_ERR_OOM, "param buffer");
    const uint64_t *zh_dev = (const uint64_t *)(p + off_zh);
    // pre-decode: resolve every operand to (kind, pointer, shift/slot, stride, immediate)
    std::vector<ZOp> prog(n_instr);
    auto decode = [&](const zxp_operand &o, uint32_t &kind, const uint64_t *&ptr, int32_t &ii, uint32_t &ld,
                      uint64_t *imm) {
        ptr = nullptr;
        ii = 0;
        ld = 0;
        imm[0] = imm[1] = imm[2] = 0;
        switch (o.kind) {
        case ZXP_TMP1: kind = DK_T1; ii = (int32_t)(o.a * 64); break;
        case ZXP_TMP3: kind = DK_T3; ii = (int32_t)((n_tmp1 + 3 * o.a) * 64); break;
        case ZXP_COL:
        case ZXP_COL3:
            kind = o.kind == ZXP_COL ? DK_C1 : DK_C3;
            ptr = sections->sec[o.a] + (uint64_t)o.b * sections->ld[o.a];
            ii = (int32_t)o.c;
            ld = (uint32_t)sections->ld[o.a];
            break;
        case ZXP_LIT: kind = DK_IMM1; imm[0] = ((uint64_t)o.a | ((uint64_t)o.b << 32)) % HP; break;
        case ZXP_PUB: kind = DK_IMM1; imm[0] = publics[o.a] % HP; break;
        case ZXP_CHAL:
            kind = DK_IMM3;
            for (int t = 0; t < 3; t++) imm[t] = challenges[3 * o.a + t] % HP;
            break;
        case ZXP_EVAL:
            kind = DK_IMM3;
            for (int t = 0; t < 3; t++) imm[t] = evals[3 * o.a + t] % HP;
            break;
        case ZXP_IMM:
            kind = o.b == 3 ? DK_IMM3 : DK_IMM1;
            for (int t = 0; t < 3; t++) imm[t] = csts[3 * o.a + t];
            break;
        case ZXP_X: kind = DK_X; break;
        case ZXP_XDIV: kind = DK_I3; ptr = xdiv; break;
        case ZXP_XDIVW: kind = DK_I3; ptr = xdivw; break;
        case ZXP_ZI: kind = DK_ZI; ptr = zh_dev; ii = (int32_t)(zh - 1); break;
        default: kind = DK_IMM1; break;
        }
    };
    std::vector<ZTerm> zterms;
    zterms.reserve(n_dot_terms);
    for (uint32_t k = 0; k < n_instr; k++) {
        ZOp &z = prog[k];
        memset(&z, 0, sizeof(z));
        z.op = pin[k].op;
        if (z.op == ZXP_DOT1 || z.op == ZXP_DOT3) {
            uint64_t c0[3] = {0, 0, 0};
            z.ia = (int32_t)zterms.size();
            for (uint32_t t = pin[k].a; t < pin[k].a + pin[k].b; t++) {
                const zxp_term &tm = terms[t];
                if (tm.src == ZXP_TERM_ONE) {
                    for (int j = 0; j < 3; j++) c0[j] = h_add(c0[j], tm.coef[j] % HP);
                    continue;
                }
                ZTerm zt;
                memset(&zt, 0, sizeof(zt));
                const zxp_operand &o = opv[tm.src];
                if (o.kind == ZXP_COL) {
                    zt.kind = DK_C1;
                    zt.ptr = sections->sec[o.a] + (uint64_t)o.b * sections->ld[o.a];
                    zt.ii = (int32_t)o.c;
                } else if (o.kind == ZXP_TMP1) {
                    zt.kind = DK_T1;
                    zt.ii = (int32_t)(o.a * 64);
                } else if (o.kind == ZXP_TMP3) {
                    zt.kind = DK_T1;
                    zt.ii = (int32_t)((n_tmp1 + 3 * o.a + tm.comp) * 64);
                } else {
                    return set_error(ZKGPU_ERR_ARG, "zxp: DOT term source kind %u", o.kind);
                }
                for (int j = 0; j < 3; j++) zxp_limbs6(tm.coef[j] % HP, zt.c[j]);
                zterms.push_back(zt);
            }
            z.ib = (int32_t)(zterms.size() - (size_t)z.ia);
            uint32_t *kl = reinterpret_cast<uint32_t *>(z.ima);  // 9 u32 over ima/imb
            for (int j = 0; j < 3; j++) {
                kl[3 * j] = (uint32_t)(c0[j] & ((1u << 22) - 1));
                kl[3 * j + 1] = (uint32_t)((c0[j] >> 22) & ((1u << 21) - 1));
                kl[3 * j + 2] = (uint32_t)(c0[j] >> 43);
            }
        } else {
            decode(opv[pin[k].a], z.ka, z.pa, z.ia, z.lda, z.ima);
            if (pin[k].op != ZXP_COPY) decode(opv[pin[k].b], z.kb, z.pb, z.ib, z.ldb, z.imb);
        }
        const uint64_t *pd;
        uint64_t dimm[3];
        decode(opv[pin[k].dst], z.kd, pd, z.id, z.ldd, dimm);
        z.pd = const_cast<uint64_t *>(pd);
        if (z.kd != DK_T1 && z.kd != DK_T3 && z.kd != DK_C1 && z.kd != DK_C3)
            return set_error(ZKGPU_ERR_ARG, "zxp: instruction %u writes a read-only operand", k);
        // a shifted store (the reference's parser opcodes 101-114 / 119 write
        // pols[off + ((i + s) % N) * stride], step3.parser.cpp) lands on row
        // (i + s) mod 2^log_dom; in a row block (no wrap-around) on local row
        // i + s, the last s of them in the halo rows (ld checked above), which
        // the caller hands to the next block's owner
    }
    if (!use_jit) {  // interpreter temporaries live in LDS
        const uint64_t slots = (uint64_t)n_tmp1 + 3ULL * n_tmp3;
        if (slots * 64 * 8 > 160 * 1024)
            return set_error(ZKGPU_ERR_ARG, "zxp: %llu temp slots exceed LDS", (unsigned long long)slots);
    }
    if ((rc = check_hip(hipMemcpyAsync(p + off_prog, prog.data(), n_instr * sizeof(ZOp), hipMemcpyHostToDevice, s),
                        "H2D")) ||
        (zterms.size() &&
         (rc = check_hip(hipMemcpyAsync(p + off_terms, zterms.data(), zterms.size() * sizeof(ZTerm),
                                        hipMemcpyHostToDevice, s),
                         "H2D"))) ||
        (rc = check_hip(hipMemcpyAsync(p + off_zh, zhv, zh * 8, hipMemcpyHostToDevice, s), "H2D")))
        return rc;
    // the sources are pageable host memory (zhv lives on this stack): the
    // uploads must complete before returning
    if ((rc = check_hip(hipStreamSynchronize(s), "zxp param upload"))) return rc;
    ZxpLaunch L;
    for (int k = 0; k < SEC_COUNT; k++) {
        L.sec[k] = sections->sec[k];
        L.ld[k] = sections->ld[k];
    }
    L.prog = (const ZOp *)(p + off_prog);
    L.terms = (const ZTerm *)(p + off_terms);
    L.n_instr = n_instr;
    L.n_tmp1 = n_tmp1;
    L.n_tmp3 = n_tmp3;
    L.logdom = log_dom;
    L.logomega = log_omega;
    L.wrap = wrap ? 1u : 0u;
    L.challenges = nullptr;
    L.publics = nullptr;
    L.evals = nullptr;
    L.xdiv = xdiv;
    L.xdivw = xdivw;
    L.zhinv = zh_dev;
    L.zhinv_mask = (uint32_t)(zh - 1);
    L.x_start = x_start % HP;
    L.bytes = alg_bytes;
    return zxp_eval(L, s);
}

int zkgpu_zxp_eval_dev(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd, uint32_t n_tmp1,
                       uint32_t n_tmp3, const zkgpu_sections *sections, uint32_t log_dom, const uint64_t *challenges,
                       const uint64_t *publics, uint32_t n_publics, const uint64_t *evals, uint32_t n_evals,
                       const uint64_t *xdiv, const uint64_t *xdivw, uint32_t extend_bits, uint64_t x_start)
{
    return zxp_eval_impl(instr, n_instr, opnd, n_opnd, n_tmp1, n_tmp3, sections, log_dom, log_dom, 1, challenges,
                         publics, n_publics, evals, n_evals, xdiv, xdivw, extend_bits, x_start);
}

int zkgpu_zxp_eval_block_dev(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd, uint32_t n_tmp1,
                             uint32_t n_tmp3, const zkgpu_sections *sections, uint32_t log_rows, uint32_t log_domain,
                             const uint64_t *challenges, const uint64_t *publics, uint32_t n_publics,
                             const uint64_t *evals, uint32_t n_evals, const uint64_t *xdiv, const uint64_t *xdivw,
                             uint32_t extend_bits, uint64_t x_start)
{
    return zxp_eval_impl(instr, n_instr, opnd, n_opnd, n_tmp1, n_tmp3, sections, log_rows, log_domain, 0, challenges,
                         publics, n_publics, evals, n_evals, xdiv, xdivw, extend_bits, x_start);
}

int zkgpu_calculate_z_block_dev(uint64_t *z, uint64_t z_ld, const uint64_t *num, uint64_t num_ld, const uint64_t *den,
                                uint64_t den_ld, uint64_t n, const uint64_t z0[3], uint64_t total[3])
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!z0 || !total) return set_error(ZKGPU_ERR_ARG, "calculate_z_block: null z0 / total");
    if (!n) {
        for (int k = 0; k < 3; k++) total[k] = z0[k] % HP;
        return 0;
    }
    const size_t words = calculate_z_scratch_words(n);
    uint64_t *scr = workspace(2, (words + 8) * sizeof(uint64_t));
    if (!scr) return ZKGPU_ERR_OOM;
    uint64_t *tot = scr + words;
    if ((rc = calculate_z(z, z_ld, num, num_ld, den, den_ld, n, z0, scr, tot, g_ctx.stream))) return rc;
    if ((rc = check_hip(hipMemcpyAsync(total, tot, 24, hipMemcpyDeviceToHost, g_ctx.stream), "D2H"))) return rc;
    return check_hip(hipStreamSynchronize(g_ctx.stream), "calculateZ sync");
}

int zkgpu_calculate_z_many_dev(const zkgpu_z_req *req, uint32_t nz, uint64_t n, int *closes)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!nz) return 0;
    if (!req || !closes) return set_error(ZKGPU_ERR_ARG, "calculate_z_many: null argument");
    if (!n) {
        for (uint32_t k = 0; k < nz; k++) closes[k] = 1;  // an empty product
        return 0;
    }
    // the requests run in stream order on one scratch; each keeps its total
    const size_t words = calculate_z_scratch_words(n);
    uint64_t *scr = workspace(2, (words + 3ULL * nz + 8) * sizeof(uint64_t));
    if (!scr) return ZKGPU_ERR_OOM;
    uint64_t *tot = scr + words;
    const uint64_t one[3] = {1, 0, 0};
    for (uint32_t k = 0; k < nz; k++)
        if ((rc = calculate_z(req[k].z, req[k].z_ld, req[k].num, req[k].num_ld, req[k].den, req[k].den_ld, n, one, scr,
                              tot + 3ULL * k, g_ctx.stream)))
            return rc;
    std::vector<uint64_t> t(3ULL * nz);
    if ((rc = check_hip(hipMemcpyAsync(t.data(), tot, t.size() * 8, hipMemcpyDeviceToHost, g_ctx.stream), "D2H")))
        return rc;
    if ((rc = check_hip(hipStreamSynchronize(g_ctx.stream), "calculateZ sync"))) return rc;
    for (uint32_t k = 0; k < nz; k++) closes[k] = (t[3 * k] == 1 && t[3 * k + 1] == 0 && t[3 * k + 2] == 0) ? 1 : 0;
    return 0;
}

int zkgpu_calculate_z_dev(uint64_t *z, uint64_t z_ld, const uint64_t *num, uint64_t num_ld, const uint64_t *den,
                          uint64_t den_ld, uint64_t n, int *closes)
{
    const uint64_t one[3] = {1, 0, 0};
    uint64_t tot[3] = {1, 0, 0};
    const int rc = zkgpu_calculate_z_block_dev(z, z_ld, num, num_ld, den, den_ld, n, one, tot);
    if (rc) return rc;
    // z[n-1] * num[n-1] / den[n-1] == 1: the product of every ratio
    if (closes) *closes = (tot[0] == 1 && tot[1] == 0 && tot[2] == 0) ? 1 : 0;
    return 0;
}

int zkgpu_evmap_dev(uint64_t *evals_out, const uint64_t *const *cols, const uint64_t *lds, const uint32_t *dims,
                    const uint32_t *primes, uint32_t n_ev, const uint64_t *lev, const uint64_t *lpev, uint64_t l_ld,
                    uint64_t n, uint32_t extend_bits)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!n_ev) return 0;
    // sub-entries: a dim-1 entry is one, a dim-3 entry three (component j,
    // weighted by X^j when the sums are combined); grouped by L (prime or not)
    // into EV_G-wide groups
    struct G {
        const uint64_t *col[8];
        uint32_t prime, sub0;
    };
    if (evmap_group_size() != sizeof(G) || evmap_group_width() != 8) return set_error(ZKGPU_ERR_ARG, "evmap group layout");
    constexpr uint32_t GW = 4;  // sub-entries per group: accumulator VGPRs vs shared limb work
    constexpr uint32_t UR = 2;  // rows per thread and iteration
    struct Sub {
        const uint64_t *col;
        uint32_t prime, which, entry;
    };
    std::vector<Sub> subs;
    for (uint32_t e = 0; e < n_ev; e++) {
        if (dims[e] != 1 && dims[e] != 3) return set_error(ZKGPU_ERR_ARG, "evmap: entry %u dim %u", e, dims[e]);
        for (uint32_t j = 0; j < dims[e]; j++) subs.push_back(Sub{cols[e] + (uint64_t)j * lds[e], primes[e] ? 1u : 0u, j, e});
    }
    std::stable_sort(subs.begin(), subs.end(), [](const Sub &a, const Sub &b) { return a.prime < b.prime; });
    std::vector<G> groups;
    std::vector<int32_t> sub_of(3 * (size_t)n_ev, -1);
    for (size_t i = 0; i < subs.size();) {
        G g;
        memset(&g, 0, sizeof(g));
        g.prime = subs[i].prime;
        g.sub0 = (uint32_t)i;
        uint32_t c = 0;
        while (c < GW && i < subs.size() && subs[i].prime == g.prime) {
            g.col[c++] = subs[i].col;
            sub_of[3 * (size_t)subs[i].entry + subs[i].which] = (int32_t)i;
            i++;
        }
        groups.push_back(g);
    }
    const uint64_t rpb = evmap_rows_per_block();
    const uint64_t nblk_ = (n + rpb - 1) / rpb;
    const size_t off_sub = (groups.size() * sizeof(G) + 15) & ~15ULL;
    const size_t off_part = (off_sub + sub_of.size() * 4 + 15) & ~15ULL;
    const size_t off_ev = off_part + subs.size() * nblk_ * 24;
    char *p = param_buf(off_ev + n_ev * 24);
    if (!p) return set_error(ZKGPU_ERR_OOM, "param buffer");
    if ((rc = check_hip(hipMemcpyAsync(p, groups.data(), groups.size() * sizeof(G), hipMemcpyHostToDevice,
                                       g_ctx.stream), "H2D")) ||
        (rc = check_hip(hipMemcpyAsync(p + off_sub, sub_of.data(), sub_of.size() * 4, hipMemcpyHostToDevice,
                                       g_ctx.stream), "H2D")) ||
        (rc = check_hip(hipStreamSynchronize(g_ctx.stream), "evmap param upload")))
        return rc;
    if ((rc = evmap_groups((uint64_t *)(p + off_ev), p, (uint32_t)groups.size(), GW, UR, (const int32_t *)(p + off_sub), n_ev,
                           (uint32_t)subs.size(), lev, lpev, l_ld, n, extend_bits, (uint64_t *)(p + off_part),
                           g_ctx.stream)))
        return rc;
    if ((rc = check_hip(hipMemcpyAsync(evals_out, p + off_ev, n_ev * 24, hipMemcpyDeviceToHost, g_ctx.stream), "D2H")))
        return rc;
    return check_hip(hipStreamSynchronize(g_ctx.stream), "evmap sync");
}

int zkgpu_xdivxsub_dev(uint64_t *xdiv, uint64_t *xdivw, const uint64_t xi[3], uint32_t n_bits, uint32_t n_bits_ext)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (n_bits_ext > TW_MAX_LOG || n_bits > n_bits_ext) return set_error(ZKGPU_ERR_ARG, "xdivxsub: bits");
    return xdivxsub(xdiv, xdivw, xi, h_w(n_bits), n_bits_ext, g_ctx.stream);
}

int zkgpu_xdivxsub_rows_dev(uint64_t *xdiv, uint64_t *xdivw, const uint64_t xi[3], uint32_t n_bits,
                            uint32_t n_bits_ext, uint64_t row0, uint64_t nrows)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (n_bits_ext > TW_MAX_LOG || n_bits > n_bits_ext) return set_error(ZKGPU_ERR_ARG, "xdivxsub_rows: bits");
    if (row0 > (1ULL << n_bits_ext) || nrows > (1ULL << n_bits_ext) - row0)
        return set_error(ZKGPU_ERR_ARG, "xdivxsub_rows: rows [%llu, +%llu) outside the domain",
                         (unsigned long long)row0, (unsigned long long)nrows);
    return xdivxsub_rows(xdiv, xdivw, xi, h_w(n_bits), n_bits_ext, row0, nrows, g_ctx.stream);
}

// F_p^3 helpers for the closed-form weights (host)
static void h3_mul(uint64_t r[3], const uint64_t a[3], const uint64_t b[3])
{
    // x^3 = x + 1
    const uint64_t c0 = h_mul(a[0], b[0]);
    const uint64_t c1 = (uint64_t)(((unsigned __int128)h_mul(a[0], b[1]) + h_mul(a[1], b[0])) % ZK_P);
    const uint64_t c2 =
        (uint64_t)(((unsigned __int128)h_mul(a[0], b[2]) + h_mul(a[1], b[1]) + h_mul(a[2], b[0])) % ZK_P);
    const uint64_t c3 = (uint64_t)(((unsigned __int128)h_mul(a[1], b[2]) + h_mul(a[2], b[1])) % ZK_P);
    const uint64_t c4 = h_mul(a[2], b[2]);
    r[0] = (uint64_t)(((unsigned __int128)c0 + c3) % ZK_P);
    r[1] = (uint64_t)(((unsigned __int128)c1 + c3 + c4) % ZK_P);
    r[2] = (uint64_t)(((unsigned __int128)c2 + c4) % ZK_P);
}

int zkgpu_lagrange_xi_rows_dev(uint64_t *lev, uint64_t *lpev, uint64_t ld, const uint64_t xi[3], uint32_t n_bits,
                               uint64_t row0, uint64_t nrows)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (n_bits > TW_MAX_LOG) return set_error(ZKGPU_ERR_ARG, "lagrange_xi_rows: bits");
    const uint64_t N = 1ULL << n_bits;
    if (row0 > N || nrows > N - row0 || (nrows && ld < nrows))
        return set_error(ZKGPU_ERR_ARG, "lagrange_xi_rows: rows [%llu, +%llu) outside the domain or ld too small",
                         (unsigned long long)row0, (unsigned long long)nrows);
    const uint64_t x[3] = {xi[0] % ZK_P, xi[1] % ZK_P, xi[2] % ZK_P};
    if (x[1] == 0 && x[2] == 0)  // xi in the base field: x_k - xi may vanish; the caller interpolates instead
        return set_error(ZKGPU_ERR_ARG, "lagrange_xi_rows: xi lies in the base field");
    // scale = (1 - xi^N) / N
    uint64_t p[3] = {1, 0, 0}, b[3] = {x[0], x[1], x[2]};
    for (uint64_t e = N; e; e >>= 1) {
        if (e & 1) h3_mul(p, p, b);
        h3_mul(b, b, b);
    }
    const uint64_t ninv = h_inv(N % ZK_P);
    const uint64_t scale[3] = {h_mul((1 + ZK_P - p[0]) % ZK_P, ninv), h_mul((ZK_P - p[1]) % ZK_P, ninv),
                               h_mul((ZK_P - p[2]) % ZK_P, ninv)};
    const uint64_t w = h_w(n_bits);
    const uint64_t wx[3] = {h_mul(x[0], w), h_mul(x[1], w), h_mul(x[2], w)};
    return xdiv_rows(lev, lpev, ld, 0, x, wx, 1, scale, n_bits, row0, nrows, g_ctx.stream);
}

int zkgpu_ext_powers_dev(uint64_t *out, uint64_t ld, const uint64_t base[3], uint64_t n)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!n) return 0;
    return ext_powers(out, ld, base, n, g_ctx.stream);
}

int zkgpu_scale_by_powers_dev(uint64_t *cols, uint64_t ld, uint32_t ncols, uint64_t n, uint64_t base)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!n || !ncols) return 0;
    if (ld < n) return set_error(ZKGPU_ERR_ARG, "scale_by_powers: ld < n");
    return scale_powers(cols, ld, ncols, n, base, g_ctx.stream);
}

int zkgpu_qsplit_dev(uint64_t *qq2, uint64_t ld2, const uint64_t *qq1, uint64_t ld1, uint64_t n, uint32_t q_deg,
                     uint64_t shift_in)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!n) return 0;
    return qsplit(qq2, ld2, qq1, ld1, n, q_deg, shift_in, 3, 3, g_ctx.stream);
}

int zkgpu_qsplit_cols_dev(uint64_t *qq2, uint64_t ld2, const uint64_t *qq1, uint64_t ld1, uint64_t n, uint32_t q_deg,
                          uint64_t shift_in, uint32_t dim, uint32_t stride)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!n || !dim) return 0;
    if (dim > stride) return set_error(ZKGPU_ERR_ARG, "qsplit_cols: dim %u > stride %u", dim, stride);
    return qsplit(qq2, ld2, qq1, ld1, n, q_deg, shift_in, dim, stride, g_ctx.stream);
}

int zkgpu_h1h2_dev(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *f, uint64_t f_ld,
                   const uint64_t *t, uint64_t t_ld, uint64_t n, uint32_t dim, uint64_t *missing_row)
{
    int rc;
    if (missing_row) *missing_row = ~0ULL;
    if ((rc = require_init())) return rc;
    if (dim != 1 && dim != 3) return set_error(ZKGPU_ERR_ARG, "h1h2: dim must be 1 or 3");
    if (n > 0x7FFFFFFFULL) return set_error(ZKGPU_ERR_ARG, "h1h2: n too large");
    if (dim == 3 && (h1_ld < n || h2_ld < n || f_ld < n || t_ld < n))
        return set_error(ZKGPU_ERR_ARG, "h1h2: ld < n");
    if (!n) return 0;
    return h1h2(h1, h1_ld, h2, h2_ld, f, f_ld, t, t_ld, n, dim, missing_row, g_ctx.stream);
}

// ---- calculateH1H2 over row-sharded f / t (include/zkgpu.h)
static int h1h2_shard_args(uint32_t dim, uint64_t n)
{
    if (dim != 1 && dim != 3) return set_error(ZKGPU_ERR_ARG, "h1h2 (sharded): dim must be 1 or 3");
    if (n > 0x7FFFFFFFULL) return set_error(ZKGPU_ERR_ARG, "h1h2 (sharded): n too large");
    return 0;
}

int zkgpu_h1h2_shard_route(uint64_t *recs, uint64_t cap, uint32_t *n_t, uint32_t *n_f, const uint64_t *f,
                           uint64_t f_ld, const uint64_t *t, uint64_t t_ld, uint64_t nrows, uint64_t row0, uint32_t dim,
                           uint32_t world)
{
    int rc;
    if ((rc = require_init()) || (rc = h1h2_shard_args(dim, nrows))) return rc;
    if (!world || !nrows) return set_error(ZKGPU_ERR_ARG, "h1h2 (sharded): empty world or block");
    if (f_ld < nrows || t_ld < nrows) return set_error(ZKGPU_ERR_ARG, "h1h2 (sharded): ld < nrows");
    if (row0 + nrows > 0xFFFFFFFFULL) return set_error(ZKGPU_ERR_ARG, "h1h2 (sharded): rows beyond 2^32");
    return h1h2_shard_route(recs, cap, n_t, n_f, f, f_ld, t, t_ld, nrows, row0, dim, world, g_ctx.stream);
}

int zkgpu_h1h2_shard_owner(uint64_t *ret, const uint64_t *recs, uint64_t nrec, uint32_t dim, uint64_t *missing_row)
{
    int rc;
    *missing_row = ~0ULL;
    if ((rc = require_init()) || (rc = h1h2_shard_args(dim, nrec))) return rc;
    return h1h2_shard_owner(ret, recs, nrec, dim, missing_row, g_ctx.stream);
}

int zkgpu_h1h2_shard_counts(uint32_t *start, uint32_t *cnt, uint64_t *total, const uint64_t *sent, const uint64_t *ret,
                            uint64_t nsent, uint64_t nrows, uint64_t row0)
{
    int rc;
    if ((rc = require_init()) || (rc = h1h2_shard_args(1, nrows))) return rc;
    if (!nrows) return set_error(ZKGPU_ERR_ARG, "h1h2 (sharded): empty block");
    return h1h2_shard_counts(start, cnt, total, sent, ret, nsent, nrows, row0, g_ctx.stream);
}

int zkgpu_h1h2_shard_deal(uint64_t *seg, uint64_t seg_ld, const uint64_t *t, uint64_t t_ld, const uint32_t *start,
                          const uint32_t *cnt, uint64_t nrows, uint32_t dim)
{
    int rc;
    if ((rc = require_init()) || (rc = h1h2_shard_args(dim, nrows))) return rc;
    if (!nrows) return 0;
    return h1h2_shard_deal(seg, seg_ld, t, t_ld, start, cnt, nrows, dim, g_ctx.stream);
}

int zkgpu_h1h2_shard_place(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *buf,
                           uint64_t buf_ld, uint64_t pos0, uint64_t len, uint64_t row0, uint32_t dim)
{
    int rc;
    if ((rc = require_init()) || (rc = h1h2_shard_args(dim, len))) return rc;
    if (len && (pos0 >> 1) < row0) return set_error(ZKGPU_ERR_ARG, "h1h2 (sharded): position before the block");
    return h1h2_shard_place(h1, h1_ld, h2, h2_ld, buf, buf_ld, pos0, len, row0, dim, g_ctx.stream);
}

int zkgpu_cols3_to_interleaved_dev(uint64_t *out, const uint64_t *cols, uint64_t ld, uint64_t n)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!n) return 0;
    return cols3_to_interleaved(out, cols, ld, n, g_ctx.stream);
}

int zkgpu_gl_merkle_open_rows_dev(uint64_t *vals_out, uint64_t *sibs_out, const uint64_t *nodes, const uint64_t *src,
                                  uint64_t ncols, uint64_t nrows, const uint64_t *idx, uint64_t nq)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (!nq) return 0;
    Ctx &c = g_ctx;
    uint32_t nlev = log2u(nrows);
    for (uint64_t q = 0; q < nq; q++)
        if (idx[q] >= nrows) return set_error(ZKGPU_ERR_ARG, "merkle_open: index out of range");
    size_t nv = nq * ncols, ns = nq * nlev * 4;
    uint64_t *d = workspace(2, (nq + nv + ns + 1) * sizeof(uint64_t));
    if (!d) return ZKGPU_ERR_OOM;
    uint64_t *didx = d, *dv = d + nq, *ds = d + nq + nv;
    if ((rc = check_hip(hipMemcpyAsync(didx, idx, nq * 8, hipMemcpyHostToDevice, c.stream), "H2D"))) return rc;
    if ((rc = merkle_open_strided(dv, ds, nodes, src, ncols, nrows, ncols, 1, didx, nq, c.stream))) return rc;
    if (nv && (rc = check_hip(hipMemcpyAsync(vals_out, dv, nv * 8, hipMemcpyDeviceToHost, c.stream), "D2H"))) return rc;
    if (ns && (rc = check_hip(hipMemcpyAsync(sibs_out, ds, ns * 8, hipMemcpyDeviceToHost, c.stream), "D2H"))) return rc;
    return check_hip(hipStreamSynchronize(c.stream), "merkle_open_rows sync");
}

// all query openings of a proof in one round trip: [indices of every request |
// vals, sibs of every request] in workspace 2, mirrored in a page-locked host
// buffer so that the upload and the download are one copy each
int zkgpu_gl_merkle_open_many(const zkgpu_open_req *req, uint32_t n)
{
    int rc;
    if ((rc = require_init())) return rc;
    Ctx &c = g_ctx;
    uint64_t ni = 0, no = 0;
    for (uint32_t k = 0; k < n; k++) {
        const zkgpu_open_req &r = req[k];
        if (r.nrows == 0 || (r.nrows & (r.nrows - 1)))
            return set_error(ZKGPU_ERR_ARG, "merkle_open_many: request %u: nrows %llu is not a power of two", k,
                             (unsigned long long)r.nrows);
        for (uint64_t q = 0; q < r.nq; q++)
            if (r.idx[q] >= r.nrows)
                return set_error(ZKGPU_ERR_ARG, "merkle_open_many: request %u: index %llu >= nrows", k,
                                 (unsigned long long)r.idx[q]);
        ni += r.nq;
        no += r.nq * (r.ncols + log2u(r.nrows) * 4ULL);
    }
    if (!ni) return 0;
    static uint64_t *pin = nullptr;
    static uint64_t pin_words = 0;
    if (pin_words < ni + no) {
        if (pin) (void)hipHostFree(pin);
        pin = nullptr;
        pin_words = 0;
        if ((rc = check_hip(hipHostMalloc((void **)&pin, (ni + no) * 8, hipHostMallocDefault), "open_many pin")))
            return rc;
        pin_words = ni + no;
    }
    uint64_t *d = workspace(2, (ni + no) * 8);
    if (!d) return ZKGPU_ERR_OOM;
    for (uint32_t k = 0, i = 0; k < n; i += req[k].nq, k++) memcpy(pin + i, req[k].idx, req[k].nq * 8);
    if ((rc = check_hip(hipMemcpyAsync(d, pin, ni * 8, hipMemcpyHostToDevice, c.stream), "open_many H2D"))) return rc;
    uint64_t io = 0, oo = ni;
    for (uint32_t k = 0; k < n; k++) {
        const zkgpu_open_req &r = req[k];
        if (!r.nq) continue;
        uint64_t *dv = d + oo, *ds = dv + r.nq * r.ncols;
        rc = r.rows ? merkle_open_strided(dv, ds, r.nodes, r.src, r.ncols, r.nrows, r.ncols, 1, d + io, r.nq, c.stream)
                    : merkle_open_cols(dv, ds, r.nodes, r.src, r.ncols, r.nrows, r.ld, d + io, r.nq, c.stream);
        if (rc) return rc;
        io += r.nq;
        oo += r.nq * (r.ncols + log2u(r.nrows) * 4ULL);
    }
    if ((rc = check_hip(hipMemcpyAsync(pin + ni, d + ni, no * 8, hipMemcpyDeviceToHost, c.stream), "open_many D2H")))
        return rc;
    if ((rc = check_hip(hipStreamSynchronize(c.stream), "open_many sync"))) return rc;
    oo = ni;
    for (uint32_t k = 0; k < n; k++) {
        const zkgpu_open_req &r = req[k];
        const uint64_t nv = r.nq * r.ncols, ns = r.nq * log2u(r.nrows) * 4ULL;
        if (nv) memcpy(r.vals_out, pin + oo, nv * 8);
        if (ns) memcpy(r.sibs_out, pin + oo + nv, ns * 8);
        oo += nv + ns;
    }
    return 0;
}

// ---------------------------------------------------------------- FRI
int zkgpu_fri_fold_dev(uint64_t *out, const uint64_t *pol, uint32_t pol_bits, uint32_t out_bits,
                       const uint64_t special_x[3], uint64_t shift_inv)
{
    int rc;
    if ((rc = require_init())) return rc;
    return fri_fold(out, pol, pol_bits, out_bits, special_x, shift_inv, g_ctx.stream);
}

int zkgpu_fri_fold_rows_dev(uint64_t *out, const uint64_t *rows, uint64_t g0, uint64_t ngroups, uint32_t pol_bits,
                            uint32_t out_bits, const uint64_t special_x[3], uint64_t shift_inv)
{
    int rc;
    if ((rc = require_init())) return rc;
    return fri_fold_rows(out, rows, g0, ngroups, pol_bits, out_bits, special_x, shift_inv, g_ctx.stream);
}

int zkgpu_fri_transpose_dev(uint64_t *aux, const uint64_t *pol, uint64_t degree, uint32_t transpose_bits)
{
    int rc;
    if ((rc = require_init())) return rc;
    return fri_transpose(aux, pol, degree, transpose_bits, g_ctx.stream);
}

}  // extern "C"

// ---------------------------------------------------------------- profiling
#include <string>
#include <vector>

namespace zk {
struct ProfRec {
    std::string name;
    hipEvent_t start, stop;
    double bytes;
};
static bool g_prof = false;
static std::vector<ProfRec> g_prof_recs;
static std::vector<hipEvent_t> g_event_pool;
static hipEvent_t g_pending_start = nullptr;

static hipEvent_t get_event()
{
    if (!g_event_pool.empty()) {
        hipEvent_t e = g_event_pool.back();
        g_event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

bool prof_on() { return g_prof; }

void prof_begin(hipStream_t s)
{
    if (!g_prof) return;
    g_pending_start = get_event();
    (void)hipEventRecord(g_pending_start, s);
}

void prof_end(const char *kernel, double bytes, hipStream_t s)
{
    if (!g_prof || !g_pending_start) return;
    hipEvent_t stop = get_event();
    (void)hipEventRecord(stop, s);
    g_prof_recs.push_back(ProfRec{kernel, g_pending_start, stop, bytes});
    g_pending_start = nullptr;
}
}  // namespace zk

extern "C" {
int zkgpu_prof_enable(int on)
{
    zk::g_prof = on != 0;
    return 0;
}

int zkgpu_prof_reset(void)
{
    (void)hipStreamSynchronize(zk::g_ctx.stream);
    for (auto &r : zk::g_prof_recs) {
        zk::g_event_pool.push_back(r.start);
        zk::g_event_pool.push_back(r.stop);
    }
    zk::g_prof_recs.clear();
    return 0;
}

int zkgpu_prof_query(const char *kernel, uint64_t *launches, double *total_ms, double *total_bytes)
{
    int rc;
    if ((rc = zk::check_hip(hipStreamSynchronize(zk::g_ctx.stream), "prof sync"))) return rc;
    uint64_t n = 0;
    double ms = 0, bytes = 0;
    for (auto &r : zk::g_prof_recs) {
        if (r.name != kernel) continue;
        float t = 0;
        if ((rc = zk::check_hip(hipEventSynchronize(r.stop), "prof event"))) return rc;
        if ((rc = zk::check_hip(hipEventElapsedTime(&t, r.start, r.stop), "prof elapsed"))) return rc;
        n++;
        ms += t;
        bytes += r.bytes;
    }
    *launches = n;
    *total_ms = ms;
    *total_bytes = bytes;
    return 0;
}

int zkgpu_prof_kernels(char *buf, uint64_t buflen)
{
    std::vector<std::string> seen;
    for (auto &r : zk::g_prof_recs) {
        bool dup = false;
        for (auto &s : seen) dup |= (s == r.name);
        if (!dup) seen.push_back(r.name);
    }
    std::string out;
    for (auto &s : seen) out += s + "\n";
    if (buflen == 0) return 0;
    size_t n = out.size() < buflen - 1 ? out.size() : buflen - 1;
    memcpy(buf, out.data(), n);
    buf[n] = 0;
    return 0;
}
// stream marks for the host prover's stage timers (no synchronisation);
// events belong to a device: a zkgpu_init on another device drops them
static hipEvent_t g_marks[ZKGPU_MARKS];
static int g_marks_dev = -1;
int zkgpu_mark(uint32_t slot)
{
    int rc;
    if ((rc = require_init())) return rc;
    if (slot >= ZKGPU_MARKS) return set_error(ZKGPU_ERR_ARG, "mark: slot %u >= %d", slot, ZKGPU_MARKS);
    if (g_marks_dev != g_ctx.device) {
        for (hipEvent_t &e : g_marks)
            if (e) {
                (void)hipEventDestroy(e);
                e = nullptr;
            }
        g_marks_dev = g_ctx.device;
    }
    if (!g_marks[slot] && (rc = check_hip(hipEventCreate(&g_marks[slot]), "mark event"))) return rc;
    return check_hip(hipEventRecord(g_marks[slot], g_ctx.stream), "mark record");
}
int zkgpu_mark_elapsed(uint32_t a, uint32_t b, double *ms)
{
    int rc;
    if (a >= ZKGPU_MARKS || b >= ZKGPU_MARKS || !g_marks[a] || !g_marks[b] || !ms)
        return set_error(ZKGPU_ERR_ARG, "mark_elapsed: slots %u / %u not recorded", a, b);
    if ((rc = check_hip(hipEventSynchronize(g_marks[b]), "mark sync"))) return rc;
    float t = 0;
    if ((rc = check_hip(hipEventElapsedTime(&t, g_marks[a], g_marks[b]), "mark elapsed"))) return rc;
    *ms = t;
    return 0;
}
}  // extern "C"
