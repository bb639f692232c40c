// Run-time compiled expression kernels for ZXP programs.
//
// The reference ships its constraint/FRI expressions as generated C++ compiled
// into the prover (src/starkpil/*/chelpers/*.step42ns.cpp, step52ns.cpp: one
// straight-line function per circuit).  This is the GPU equivalent: the
// compiled program (csrc/zxp_compile.cpp: fused DOT instructions, SSA temps
// packed into slots) is printed as one straight-line HIP kernel -- temporaries
// in registers, every column read a coalesced load the compiler can schedule
// freely, column stores deferred to the end of the row -- and compiled for
// gfx950 with hiprtc on first use.  Only the program STRUCTURE is in the
// source (column slots, row shifts, table offsets); challenge-dependent
// values (DOT coefficient limbs, F_p^3 constants) and pointers are kernel
// inputs, so one compiled kernel serves every proof of a circuit (cached per
// process by source text).  csrc/gl_device.hpp is embedded verbatim, so the
// field arithmetic is the same code the interpreter (k_zxp_eval) runs.
//
// Unsupported shapes (a program that reads a column it writes at a row shift
// it did not write first) return 1 and the caller runs the interpreter.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>
#include <utime.h>

#include <chrono>
#include <cctype>
#include <charconv>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <array>
#include <map>
#include <set>
#include <mutex>
#include <chrono>
#include <string>
#include <unordered_map>
#include <vector>

#include "zkgpu_internal.hpp"
#include "zxp_segment.hpp"

#include <algorithm>
#include <atomic>
#include <functional>
#include <thread>

namespace zk {

static const char *k_gl_device_src =
#include "../build/gl_device_src.inc"
    ;

namespace {

constexpr int JIT_THREADS = 256;

// column term of a looped DOT (device table; layout shared with k_kernel_head)
struct JitTerm {
    const uint64_t *ptr;
    int64_t sh;
    uint32_t c[3][6];
    uint32_t pad[2];
};
static_assert(sizeof(JitTerm) == 96, "JitTerm");

struct JitParams {
    const uint64_t *const *cp;  // column base pointers (slot j)
    const uint64_t *kc;         // F_p / F_p^3 constants
    const uint32_t *kl;         // DOT limbs (unrolled terms)
    const JitTerm *zt;          // DOT column terms (looped)
    const uint64_t *xdiv, *xdivw, *zh, *tw_lo, *tw_hi;
    uint64_t x_start, rmask;
    uint32_t logdom, logomega, zmask;
    uint32_t nkl;  // limb words staged in LDS (0: read from p.kl)
    uint32_t one;  // always 1: the uniform branch that closes each code block (compile time)
};

// DOT limb tables up to this size are staged in LDS per workgroup: read from
// there, the straight-line terms' constants do not compete for the 106 SGPRs
// (scalar loads of every term's limbs hoisted by the scheduler spill SGPRs
// into VGPR lanes -- thousands of v_readlane/v_writelane per row).
constexpr size_t JIT_KL_LDS_MAX = 48 * 1024;
constexpr int JIT_KCHUNK = 1024;  // words per LDS limb chunk (256 threads x 16 bytes)

const char *k_kernel_head = R"(
using namespace zk;
struct JitTerm {
    const uint64_t *ptr;
    int64_t sh;
    uint32_t c[3][6];
    uint32_t pad[2];
};
struct JitParams {
    const uint64_t *const *cp;
    const uint64_t *kc;
    const uint32_t *kl;
    const JitTerm *zt;
    const uint64_t *xdiv, *xdivw, *zh, *tw_lo, *tw_hi;
    uint64_t x_start, rmask;
    uint32_t logdom, logomega, zmask;
    uint32_t nkl;
    uint32_t one;
};
// long column runs of a DOT: a loop over table terms, ZKJIT_UNROLL loads in flight
template <int D>
__device__ __forceinline__ void dot_cols(Dot3 &d0, Dot3 &d1, Dot3 &d2, const JitTerm *t, int n, uint64_t i,
                                         uint64_t m)
{
    constexpr int U = ZKJIT_UNROLL;
    int k = 0;
    for (; k + U <= n; k += U) {
        uint64_t a[U];
#pragma unroll
        for (int u = 0; u < U; u++) a[u] = gload(t[k + u].ptr + ((i + (uint64_t)t[k + u].sh) & m));
#pragma unroll
        for (int u = 0; u < U; u++) {
            d0.term(a[u], t[k + u].c[0]);
            if (D == 3) {
                d1.term(a[u], t[k + u].c[1]);
                d2.term(a[u], t[k + u].c[2]);
            }
        }
    }
    for (; k < n; k++) {
        const uint64_t a = gload(t[k].ptr + ((i + (uint64_t)t[k].sh) & m));
        d0.term(a, t[k].c[0]);
        if (D == 3) {
            d1.term(a, t[k].c[1]);
            d2.term(a, t[k].c[2]);
        }
    }
}
// one 16-byte slice of a limb chunk per thread (256 threads: 1024 words)
__device__ __forceinline__ uint4 kpre(const uint32_t *kl, size_t lo)
{
    return *(const __attribute__((address_space(1))) uint4 *)(kl + lo + 4 * threadIdx.x);
}
__device__ __forceinline__ void kput(uint32_t *dst, uint4 v) { *(uint4 *)(dst + 4 * threadIdx.x) = v; }
__device__ __forceinline__ uint64_t gload_o(const uint64_t *base, uint32_t byte_off)
{
    return *(const gu64_t *)((const char *)base + byte_off);
}
__device__ __forceinline__ uint64_t zk_cs(uint64_t *slot, uint64_t v)
{
    *slot = v;
    return v;
}
__device__ __forceinline__ int zk_one()
{
    int c;
    asm volatile("s_mov_b32 %0, 1" : "=s"(c));
    return c;
}
extern "C" __global__ void __launch_bounds__(256) ZKJIT_WAVES zxp_jit(const JitParams p)
{
#if ZKJIT_KL_LDS
    extern __shared__ __attribute__((aligned(16))) uint32_t kls[];
    for (uint32_t w = threadIdx.x; w < p.nkl; w += 256) kls[w] = p.kl[w];
    const uint32_t *K = kls;
#else
    const uint32_t *K = p.kl;
#endif
    const JitTerm *ZT = p.zt;  // (in LDS: measured slower, 9.0 -> 11.4 ms for step52ns)
#if ZKJIT_KL_LDS
    __syncthreads();
#endif
    // ZKJIT_ROWS rows per thread: i_r = ib_ + r * S_ (each row set is
    // contiguous over the lanes, so every column load stays coalesced)
    const uint64_t S_ = (1ULL << p.logdom) / ZKJIT_ROWS;
#if ZKJIT_KL_CHUNK
    // limb chunks staged in LDS per code block (workgroup barriers: every
    // thread stays to the end, rows past the domain only skip the stores)
    const uint64_t i_ = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live_ = i_ < S_;
    const uint64_t ib_ = live_ ? i_ : 0;
    __shared__ __attribute__((aligned(16))) uint32_t kbuf[2 * ZKJIT_KL_CHUNK];
    uint4 pf_;  // the next chunk, in flight (zxp_jit_source chunk_head)
    kput(kbuf, kpre(p.kl, 0));
    __syncthreads();
#else
    const uint64_t ib_ = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (ib_ >= S_) return;
#endif
    const uint64_t m = p.rmask;
#ifdef ZK_CP_AS
#define CPTR(j) ((uint64_t *)(((const ZK_CP_AS uint64_t *)p.cp)[j]))
#else
#define CPTR(j) (const_cast<uint64_t *>(p.cp[j]))
#endif
// a column read: 32-bit byte offset from the column's (scalar) base, so the
// load takes the global_load saddr form -- one offset register per row shift
// shared by every column, no 64-bit address per load (domains <= 2^28 rows,
// api.hip use_jit)
#if ZKJIT_SADDR
const uint32_t m32_ = (uint32_t)m;
#define C(j, sh, ii) gload_o(CPTR(j), (((uint32_t)(ii) + (uint32_t)(sh)) & m32_) << 3)
#else
#define C(j, sh, ii) gload(CPTR(j) + ((ii + (uint64_t)(sh)) & m))
#endif
#if ZKJIT_LCACHE
    // compiler-managed column cache (lds_column_cache): slot s of this lane
    // (ZKJIT_ROWS rows per thread: slot s of row r at (s ROWS + r))
    __shared__ uint64_t zkc[ZKJIT_LCACHE * ZKJIT_ROWS * 256];
    uint64_t *const zkc_ = zkc + threadIdx.x;
#define LC(s, r) (zkc_[((s) * ZKJIT_ROWS + (r)) * 256])
#define CS(j, sh, ii, s, r) zk_cs(zkc_ + ((s) * ZKJIT_ROWS + (r)) * 256, C(j, sh, ii))
#endif
// scratch columns of a segmented program (csrc/zxp_segment.hpp) are stored
// where the value is defined, not deferred to the end of the row
#if ZKJIT_KL_CHUNK
#define ZK_ST(j, v, ii) do { if (live_) gstore_out(CPTR(j) + ii, gl_canon(v)); } while (0)
#define ZK_STS(j, v, ii, sh) do { if (live_) gstore_out(CPTR(j) + ((ii + (uint64_t)(int64_t)(sh)) & m), gl_canon(v)); } while (0)
#else
#define ZK_ST(j, v, ii) gstore_out(CPTR(j) + ii, gl_canon(v))
#define ZK_STS(j, v, ii, sh) gstore_out(CPTR(j) + ((ii + (uint64_t)(int64_t)(sh)) & m), gl_canon(v))
#endif
// a global limb table is re-based in every code block (an opaque copy of K):
// with thousands of loads off one base register, SIFoldOperands dominated
// the compile (48 s of 100 for step3prev)
#if ZKJIT_KL_LDS
#define ZK_KREFRESH
#else
#define ZK_KREFRESH asm volatile("" : "+s"(K));
#endif
)";

void appendf(std::string &s, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (n >= (int)sizeof(buf)) {
        std::vector<char> big(n + 1);
        va_start(ap, fmt);
        vsnprintf(big.data(), big.size(), fmt, ap);
        va_end(ap);
        s += big.data();
    } else {
        s += buf;
    }
}

// decimal text without the printf machinery (the per-term lines below are
// ~10 K appends per segment: vsnprintf was ~60 % of a segment's source time)
inline void app_num(std::string &s, uint64_t v)
{
    char b[24];
    const auto r = std::to_chars(b, b + sizeof(b), v);
    s.append(b, r.ptr);
}

// one DOT term's line: D<dot>_j`.term_al(<val>, K + <kt + 8 j>) for the
// components of the accumulator (the same text appendf wrote)
inline void app_term(std::string &s, const std::string &val, uint32_t dot, size_t kt, bool three)
{
    if (three) {
        s += "{ const uint64_t v_ = ";
        s += val;
        for (int j = 0; j < 3; j++) {
            s += j ? " D" : "; D";
            app_num(s, dot);
            s += j == 0 ? "_0`.term_al(v_, K + " : j == 1 ? "_1`.term_al(v_, K + " : "_2`.term_al(v_, K + ";
            app_num(s, kt + 8 * (size_t)j);
            s += ");";
        }
        s += " }\n";
    } else {
        s += 'D';
        app_num(s, dot);
        s += "_0`.term_al(";
        s += val;
        s += ", K + ";
        app_num(s, kt);
        s += ");\n";
    }
}

struct Expr {
    std::string e;
    int dim;
};

struct Cache {
    std::mutex mu;
    std::unordered_map<std::string, hipFunction_t> fn;
};
Cache &cache()
{
    static Cache c;
    return c;
}

// grow-only device buffer for the per-launch tables (in_use: the event after
// the last kernels that read it)
char *jit_buf(size_t bytes, hipEvent_t in_use)
{
    static char *buf = nullptr;
    static size_t cap = 0;
    if (bytes > cap) {
        if (in_use) (void)hipEventSynchronize(in_use);
        if (buf) (void)hipFree(buf);
        buf = nullptr;
        cap = 0;
        if (hipMalloc((void **)&buf, bytes) != hipSuccess) return nullptr;
        cap = bytes;
    }
    return buf;
}

// hiprtc: source -> gfx950 code object (no GPU needed)
int rtc_compile(const std::string &src, std::vector<char> &code)
{
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "zxp_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return set_error(ZKGPU_ERR_ARG, "zxp jit: hiprtcCreateProgram failed");
    // LDS-staged limb tables compile at -O2: the load/store vectorizer merges
    // each term's limb reads into 16+8-byte loads (-O1 does not run it).
    // Otherwise -O1 (-O2 is no faster there: the scheduler hoists more scalar
    // loads, e.g. step42ns without LDS 14.1 -> 16.7 ms).  Compile time is about
    // the same.
    const bool klds = src.find("#define ZKJIT_KL_LDS 1") != std::string::npos;
    const char *olev = klds ? "-O2" : "-O1";
    // The GCN scheduler's re-scheduling stages (unclustered high-pressure and
    // clustered low-occupancy) re-run the scheduler over every region and
    // doubled the compile time of the large programs; register pressure is
    // already bounded by the ZXP scheduler (csrc/zxp_compile.cpp), so they
    // are off for them.
    // Small programs keep them: there they lower register pressure (config-4
    // quotient 17.2 -> 15.2 ms, FRI polynomial 10.4 -> 9.1 ms at 2^23) and
    // cost little compile time.
    const bool resched = src.find("#define ZKJIT_SPLIT 1") == std::string::npos;
    std::vector<const char *> opts = {"--offload-arch=gfx950", olev, "-std=c++17"};
    if (!resched) {
        opts.push_back("-mllvm");
        opts.push_back("-amdgpu-disable-unclustered-high-rp-reschedule=1");
        opts.push_back("-mllvm");
        opts.push_back("-amdgpu-disable-clustered-low-occupancy-reschedule=1");
    }
    const hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (r != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(prog, &ls);
        std::string log(ls + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        return set_error(ZKGPU_ERR_ARG, "zxp jit: hiprtc compile failed: %.300s", log.c_str());
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.resize(cs);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return cs ? 0 : set_error(ZKGPU_ERR_ARG, "zxp jit: empty code object");
}

// On-disk code-object cache: a program's kernel depends only on its
// structure (the source text) and the compiler, so compiled objects are kept
// in ZKGPU_JIT_CACHE (default: <libzkgpu dir>/../jitcache, created on demand;
// "0" disables) under a hash of source + options + hiprtc version.  build()
// fills it ahead of time for the known circuits (the reference ships its
// expression code compiled, chelpers/*.cpp).
static std::string cache_dir()
{
    static const std::string dir = [] {
        const char *e = getenv("ZKGPU_JIT_CACHE");
        if (e) return std::string(strcmp(e, "0") ? e : "");
        Dl_info info;
        if (dladdr((void *)&cache_dir, &info) && info.dli_fname) {
            std::string so = info.dli_fname;
            const size_t sl = so.rfind('/');
            if (sl != std::string::npos) return so.substr(0, sl) + "/../jitcache";
        }
        return std::string();
    }();
    return dir;
}

static std::string cache_key(const std::string &src)
{
    int major = 0, minor = 0;
    hiprtcVersion(&major, &minor);
    uint64_t h1 = 1469598103934665603ULL, h2 = 0x9E3779B97F4A7C15ULL;
    auto mix = [&](const char *p, size_t n) {
        for (size_t i = 0; i < n; i++) {
            h1 = (h1 ^ (uint8_t)p[i]) * 1099511628211ULL;
            h2 = (h2 + (uint8_t)p[i]) * 0xBF58476D1CE4E5B9ULL;
            h2 ^= h2 >> 29;
        }
    };
    mix(src.data(), src.size());
    char opt[160];
    // ("opt- resched-": the compile options are a function of the source,
    // which is hashed above; the text keeps the keys of existing entries)
    snprintf(opt, sizeof(opt), "hiprtc%d.%d hip%d gfx950 opt- resched-", major, minor, (int)HIP_VERSION);
    mix(opt, strlen(opt));
    char key[64];
    snprintf(key, sizeof(key), "zxp_%016llx%016llx.co", (unsigned long long)h1, (unsigned long long)h2);
    return key;
}

// On-disk entry: "ZKJITCO2", u32 key length, key (cache_key: hash of source,
// options, hiprtc / HIP versions, target), u64 object length, object.  A file
// that does not carry this exact key and a complete ELF object is a miss.
static const char JIT_CO_MAGIC[8] = {'Z', 'K', 'J', 'I', 'T', 'C', 'O', '2'};

static bool cache_load(const std::string &src, std::vector<char> &code)
{
    const std::string dir = cache_dir();
    if (dir.empty()) return false;
    const std::string key = cache_key(src);
    FILE *f = fopen((dir + "/" + key).c_str(), "rb");
    if (!f) return false;
    char magic[8];
    uint32_t kn = 0;
    uint64_t n = 0;
    bool ok = fread(magic, 1, 8, f) == 8 && !memcmp(magic, JIT_CO_MAGIC, 8) && fread(&kn, 4, 1, f) == 1 &&
              kn == key.size();
    if (ok) {
        std::string k2(kn, '\0');
        ok = fread(&k2[0], 1, kn, f) == kn && k2 == key && fread(&n, 8, 1, f) == 1 && n > 4 && n < (1ULL << 32);
    }
    if (ok) {
        code.resize(n);
        ok = fread(code.data(), 1, n, f) == n && fgetc(f) == EOF && !memcmp(code.data(), "\x7f" "ELF", 4);
    }
    fclose(f);
    if (ok) utime((dir + "/" + key).c_str(), nullptr);  // in use: tools/jit_prebuild.py --prune keeps it
    return ok;
}

static void cache_store(const std::string &src, const std::vector<char> &code)
{
    const std::string dir = cache_dir();
    if (dir.empty()) return;
    mkdir(dir.c_str(), 0775);
    const std::string key = cache_key(src);
    const std::string path = dir + "/" + key, tmp = path + ".tmp" + std::to_string(getpid());
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) return;
    const uint32_t kn = (uint32_t)key.size();
    const uint64_t n = code.size();
    const bool ok = fwrite(JIT_CO_MAGIC, 1, 8, f) == 8 && fwrite(&kn, 4, 1, f) == 1 && fwrite(key.data(), 1, kn, f) == kn &&
                    fwrite(&n, 8, 1, f) == 1 && fwrite(code.data(), 1, n, f) == n;
    fclose(f);
    if (ok) rename(tmp.c_str(), path.c_str());
    else unlink(tmp.c_str());
}

// source -> code object: the disk cache, else hiprtc (and fill the cache);
// *cached tells which
int code_object(const std::string &src, std::vector<char> &code, bool *cached = nullptr)
{
    if (cached) *cached = false;
    if (cache_load(src, code)) {
        if (cached) *cached = true;
        return 0;
    }
    int rc;
    static const bool log = getenv("ZKGPU_JIT_LOG") && atoi(getenv("ZKGPU_JIT_LOG"));
    const auto t0 = std::chrono::steady_clock::now();
    if ((rc = rtc_compile(src, code))) return rc;
    cache_store(src, code);
    if (log)  // cache misses (tools/jit_prebuild.py fills the cache ahead of time)
        fprintf(stderr, "[zkgpu jit] cache miss: %s compiled in %.1f s\n", cache_key(src).c_str(),
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    return 0;
}

}  // namespace

// Limb tables of at least JIT_KL_LDS_MIN words are staged in LDS.  Measured
// on the config-4 STARK at 2^23:
// step42ns (4.1 K words) 14.1 -> 12.4 ms; step52ns (0.4 K words) is
// 9.2 -> 14.4 ms with LDS (its VGPRs go 74 -> 198), so small tables stay on
// scalar loads.
constexpr size_t JIT_KL_LDS_MIN = 1024;
static bool jit_kl_lds(size_t nkl)
{
    if (!nkl || nkl * 4 > JIT_KL_LDS_MAX) return false;
    return nkl >= JIT_KL_LDS_MIN;
}

// Rows per thread of a compiled kernel: one.  (With 2 rows each
// wave-uniform limb read from LDS, column pointer and instruction serves 128
// rows and two independent chains hide each other's load latency -- measured
// equal to 1 row at twice the occupancy on the zkEVM-sized quotient, 0.557 vs
// 0.547 s at 2^24 rows; the generator keeps the row expansion.)
static uint32_t jit_rows(bool) { return 1; }

// every line holding a ` is written once per row r (` -> _r, ~ -> r)
static std::string expand_rows(const std::string &text, uint32_t rows)
{
    std::string out;
    out.reserve(text.size() * rows);
    size_t pos = 0;
    while (pos < text.size()) {
        size_t eol = text.find('\n', pos);
        if (eol == std::string::npos) eol = text.size() - 1;
        const size_t len = eol + 1 - pos;
        if (memchr(text.data() + pos, '`', len) == nullptr) {
            out.append(text, pos, len);
        } else {
            for (uint32_t r = 0; r < rows; r++) {
                // runs between the marks appended whole (a line is ~50-100 chars)
                size_t k = pos;
                while (k <= eol) {
                    size_t e = k;
                    while (e <= eol && text[e] != '`' && text[e] != '~') e++;
                    out.append(text, k, e - k);
                    if (e > eol) break;
                    if (text[e] == '`') out += '_';
                    out += (char)('0' + r);
                    k = e + 1;
                }
            }
        }
        pos = eol + 1;
    }
    return out;
}

// Segment kernels (round 6, VERDICT r5 "next" 4):
// 512-byte code blocks, up to 16 LDS cache slots per lane (LDS budget
// 160 KB / waves per workgroup, 4 waves per SIMD) and the software prefetch
// below (16 loads, one block ahead).  zkEVM-shaped quotient at 2^24 rows:
// 49.9 -> 56.1 Mrow/s (r06_seg_ab.json).  A/B switch:
// ZKGPU_ZXP_SEG_AB="waves,slots,prefetch[,block bytes[,blocks ahead]]"
// (4,12,0,1024,1 = the round-5 segments).
struct SegAb {
    uint32_t waves = 0, slots = 0, prefetch = 0, block = 0, dist = 0;  // block / dist: 0 = the default
};
static const SegAb &seg_ab()
{
    static const SegAb c = [] {
        SegAb v;
        if (const char *e = getenv("ZKGPU_ZXP_SEG_AB")) {
            if (sscanf(e, "%u,%u,%u,%u,%u", &v.waves, &v.slots, &v.prefetch, &v.block, &v.dist) < 3 || v.waves > 8)
                v = SegAb();
        }
        return v;
    }();
    return c;
}

// Software prefetch across code blocks (the SEG_AB experiment): the first
// `pf` global column reads of every code block are issued at the start of the
// block before it, into per-row registers (zpf<k>`), and read from there --
// a column load then has a whole code block (~1 KB of source) to arrive
// instead of the compiler's in-block scheduling window.  Loads stay
// in flight across __syncthreads (it waits for LDS only).  Columns the kernel
// stores to are never prefetched; a cached read (CS) keeps its slot store.
// Returns the number of prefetch registers.
static uint32_t prefetch_blocks(std::string &body, uint32_t pf, uint32_t dist = 1)
{
    static const std::string head = "if (zk_one()) {\n";
    std::vector<size_t> starts;
    for (size_t q = body.find(head); q != std::string::npos; q = body.find(head, q + head.size()))
        starts.push_back(q + head.size());
    if (starts.size() < 2 || !pf) return 0;
    auto ident = [](char c) {
        return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
    };
    auto num = [&](size_t &q, int64_t &v) {
        const char *b = body.c_str() + q;
        char *e;
        v = strtoll(b, &e, 10);
        if (e == b) return false;
        q += (size_t)(e - b);
        return true;
    };
    std::set<int64_t> stored;
    for (size_t q = body.find("ZK_ST"); q != std::string::npos; q = body.find("ZK_ST", q + 5)) {
        size_t t = q + (body.compare(q, 7, "ZK_STS(") == 0 ? 7 : body.compare(q, 6, "ZK_ST(") == 0 ? 6 : 0);
        int64_t j;
        if (t > q && num(t, j)) stored.insert(j);
    }
    struct Edit {
        size_t pos, len;
        std::string text;
    };
    std::vector<Edit> edits;  // replacements and insertions, by position
    uint32_t n = 0;
    for (size_t b = 1; b < starts.size(); b++) {
        const size_t lo = starts[b], hi = b + 1 < starts.size() ? starts[b + 1] - head.size() : body.size();
        std::string loads;
        uint32_t taken = 0;
        for (size_t q = lo; q < hi && taken < pf; q++) {
            if (body[q] != 'C' || ident(body[q - 1])) continue;
            const bool cs = body.compare(q, 3, "CS(") == 0;
            if (!cs && body.compare(q, 2, "C(") != 0) continue;
            size_t t = q + (cs ? 3 : 2);
            int64_t j, sh, slot = 0;
            if (!num(t, j) || body[t] != ',') continue;
            t++;
            if (!num(t, sh) || body.compare(t, 3, ",i`") != 0) continue;
            t += 3;
            if (cs) {
                if (body[t] != ',') continue;
                t++;
                if (!num(t, slot) || body.compare(t, 3, ",~)") != 0) continue;
                t += 3;
            } else {
                if (body[t] != ')') continue;
                t++;
            }
            if (stored.count(j)) continue;
            std::string var = "zpf";
            app_num(var, n);
            var += '`';
            loads += var + " = C(";
            loads += std::to_string(j) + "," + std::to_string(sh) + ",i`);\n";
            edits.push_back({q, t - q, cs ? "CSV(" + var + "," + std::to_string(slot) + ",~)" : var});
            n++;
            taken++;
        }
        if (!loads.empty()) edits.push_back({starts[b >= dist ? b - dist : 0], 0, loads});
    }
    std::stable_sort(edits.begin(), edits.end(), [](const Edit &x, const Edit &y) { return x.pos < y.pos; });
    std::string out;
    out.reserve(body.size() + n * 40);
    size_t at = 0;
    for (const Edit &e : edits) {
        out.append(body, at, e.pos - at);
        out += e.text;
        at = e.pos + e.len;
    }
    out.append(body, at, std::string::npos);
    body.swap(out);
    return n;
}

// Compiler-managed LDS column cache for block-split programs.  A large
// program's kernel is HBM-bound on re-reads: it loads a column again at every
// use, and a re-read hits the 4 MB L2 of an XCD only within ~16 columns (512
// waves x 512 bytes per column in flight).  The whole read
// sequence is known here, so each lane keeps up to `slots` column values in
// LDS chosen by Belady's rule (on a miss, evict the value whose next read is
// furthest away, or bypass when the new value's next read is further still):
// a read of a cached value becomes an LDS read, LC(s), and a read that enters
// the cache stores its value as it loads it, CS(..., s).  The body is
// rewritten textually: every column read is a C(j,sh,i`) token, in emission
// order, one statement per line.  Within a line the operand evaluation order
// is unspecified, so a slot read or filled on a line is not evicted on that
// line.  Columns the kernel stores to are never cached.  Reads within `gap`
// reads of the previous one are left to the L1/L2.  Returns the number of
// cached reads (LDS hits).
static size_t lds_column_cache(std::string &body, int slots, int gap)
{
    struct Rd {
        size_t pos, len;
        uint64_t key;
        uint32_t line;
    };
    std::vector<Rd> rd;
    std::set<uint32_t> stored;
    auto ident = [](char c) {
        return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
    };
    auto num = [&](size_t &q, int64_t &v) {
        const char *b = body.c_str() + q;
        char *e;
        v = strtoll(b, &e, 10);
        if (e == b) return false;
        q += (size_t)(e - b);
        return true;
    };
    uint32_t line = 0;
    const char *bp = body.data();
    const size_t bn = body.size();
    for (size_t q = 0; q < bn; q++) {
        const char ch = bp[q];
        if (ch == '\n') {
            line++;
            continue;
        }
        if (ch != 'C' && ch != 'Z') continue;
        if (q > 0 && ident(bp[q - 1])) continue;
        if (ch == 'C' && body.compare(q, 2, "C(") == 0) {
            size_t t = q + 2;
            int64_t j, sh;
            if (!num(t, j) || body[t] != ',') continue;
            t++;
            if (!num(t, sh) || body.compare(t, 4, ",i`)") != 0) continue;
            rd.push_back({q, t + 4 - q, ((uint64_t)(uint32_t)j << 32) | (uint32_t)(int32_t)sh, line});
        } else if (ch == 'Z' && (body.compare(q, 6, "ZK_ST(") == 0 || body.compare(q, 7, "ZK_STS(") == 0)) {
            size_t t = q + (body[q + 5] == 'S' ? 7 : 6);
            int64_t j;
            if (num(t, j)) stored.insert((uint32_t)j);
        }
    }
    const uint64_t INF = ~0ULL;
    std::vector<uint64_t> nx(rd.size(), INF);
    {
        std::unordered_map<uint64_t, size_t> last;
        last.reserve(rd.size());
        for (size_t r = rd.size(); r-- > 0;) {
            auto it = last.find(rd[r].key);
            if (it != last.end()) nx[r] = it->second;
            last[rd[r].key] = r;
        }
    }
    std::vector<uint64_t> slot_key(slots, INF), slot_nu(slots, INF);
    std::unordered_map<uint64_t, int> where;
    std::vector<int> act(rd.size(), -1), hit(rd.size(), 0);
    std::vector<uint32_t> pinned_line(slots, UINT32_MAX);
    size_t hits = 0;
    for (size_t r = 0; r < rd.size(); r++) {
        const Rd &x = rd[r];
        if (stored.count((uint32_t)(x.key >> 32))) continue;
        auto it = where.find(x.key);
        if (it != where.end()) {
            const int sl = it->second;
            act[r] = sl;
            hit[r] = 1;
            hits++;
            pinned_line[sl] = x.line;
            slot_nu[sl] = nx[r];
            if (nx[r] == INF) {  // last read: the slot is free again
                where.erase(it);
                slot_key[sl] = INF;
            }
            continue;
        }
        if (nx[r] == INF || nx[r] - r <= (uint64_t)gap) continue;
        int v = -1;
        for (int sl = 0; sl < slots; sl++) {
            if (pinned_line[sl] == x.line) continue;
            if (slot_key[sl] == INF) {
                v = sl;
                break;
            }
            if (v < 0 || slot_nu[sl] > slot_nu[v]) v = sl;
        }
        if (v < 0 || (slot_key[v] != INF && slot_nu[v] <= nx[r])) continue;  // bypass
        if (slot_key[v] != INF) where.erase(slot_key[v]);
        slot_key[v] = x.key;
        slot_nu[v] = nx[r];
        where[x.key] = v;
        pinned_line[v] = x.line;
        act[r] = v;
    }
    if (!hits) return 0;
    std::string out;
    out.reserve(body.size() + rd.size() * 4);
    size_t at = 0;
    for (size_t r = 0; r < rd.size(); r++) {
        if (act[r] < 0) continue;
        out.append(body, at, rd[r].pos - at);
        if (hit[r]) {  // (~: the row of the line, expand_rows)
            out += "LC(";
            app_num(out, (uint64_t)act[r]);
            out += ",~)";
        } else {
            out += "CS(";
            out.append(body, rd[r].pos + 2, rd[r].len - 3);
            out += ',';
            app_num(out, (uint64_t)act[r]);
            out += ",~)";
        }
        at = rd[r].pos + rd[r].len;
    }
    out.append(body, at, std::string::npos);
    body.swap(out);
    return hits;
}

int zxp_jit_build_source(const ZxpJitIn &in, std::string &src, std::vector<const uint64_t *> &cp,
                         std::vector<uint64_t> &kc, std::vector<uint32_t> &kl, std::vector<JitTerm> &zt)
{
    const zkgpu_sections *S = in.sections;
    auto col_ptr = [&](uint32_t sec, uint32_t col) -> const uint64_t * {
        if (sec == ZXP_SEC_SCRATCH) return in.scratch + (uint64_t)col * in.scratch_ld;
        return S->sec[sec] + (uint64_t)col * S->ld[sec];
    };
    // (section, col) -> cp slot: a flat table per section (a segment looks up
    // ~10^4 column reads), a map for out-of-table indices
    std::vector<std::vector<uint32_t>> slot_of(ZXP_SEC_SCRATCH + 1);
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> slot_far;
    auto col_slot = [&](uint32_t sec, uint32_t col) -> uint32_t {
        if (sec <= ZXP_SEC_SCRATCH && col < (1u << 20)) {
            std::vector<uint32_t> &v = slot_of[sec];
            if (col >= v.size()) v.resize(col + 1, UINT32_MAX);
            if (v[col] == UINT32_MAX) {
                cp.push_back(col_ptr(sec, col));
                v[col] = (uint32_t)cp.size() - 1;
            }
            return v[col];
        }
        auto key = std::make_pair(sec, col);
        auto it = slot_far.find(key);
        if (it != slot_far.end()) return it->second;
        cp.push_back(col_ptr(sec, col));
        return slot_far[key] = (uint32_t)cp.size() - 1;
    };
    // Columns the program reads (any shift): a written column it never reads
    // is stored where the value is assigned (the compiled program forwards
    // every read of a cell the row wrote, zxp_compile.cpp); a written column
    // it also reads keeps its value in a register w<r> stored at the end of
    // the row, landing on row (i + shift) & m (reads before the write see the
    // old value).  Immediate stores keep the stage-3 programs' ~300 written
    // cells out of the registers.
    std::set<std::pair<uint32_t, uint32_t>> read_cols;
    {
        auto note = [&](uint32_t o) {
            if (o >= in.n_opnd) return;
            const zxp_operand &x = in.opnd[o];
            if (x.kind == ZXP_COL || x.kind == ZXP_COL3)
                for (uint32_t c = 0; c < (x.kind == ZXP_COL3 ? 3u : 1u); c++) read_cols.insert({x.a, x.b + c});
        };
        for (uint32_t k = 0; k < in.n_instr; k++) {
            const zxp_instr &I = in.ins[k];
            if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
                for (uint32_t t = I.a; t < I.a + I.b; t++)
                    if (in.terms[t].src != ZXP_TERM_ONE) note(in.terms[t].src);
            } else {
                note(I.a);
                if (I.op != ZXP_COPY) note(I.b);
            }
        }
    }
    auto store_now = [&](uint32_t sec, uint32_t col) {
        return sec != ZXP_SEC_SCRATCH && !read_cols.count({sec, col});
    };
    std::map<std::pair<uint32_t, int32_t>, uint32_t> wreg;
    std::vector<std::pair<uint32_t, int32_t>> wcell;  // register -> (slot, shift)
    std::vector<uint8_t> written_any;                  // per slot, at any shift
    for (uint32_t k = 0; k < in.n_instr; k++) {
        const zxp_operand &d = in.opnd[in.ins[k].dst];
        if ((d.kind == ZXP_COL || d.kind == ZXP_COL3) && d.a != ZXP_SEC_SCRATCH && !store_now(d.a, d.b))
            for (uint32_t c = 0; c < (d.kind == ZXP_COL3 ? 3u : 1u); c++) {
                const uint32_t j = col_slot(d.a, d.b + c);
                const auto key = std::make_pair(j, (int32_t)d.c);
                if (!wreg.count(key)) {
                    wreg[key] = (uint32_t)wcell.size();
                    wcell.push_back(key);
                }
                if (j >= written_any.size()) written_any.resize(j + 1, 0);
                written_any[j] = 1;
            }
    }
    auto is_written = [&](uint32_t j) { return j < written_any.size() && written_any[j]; };
    std::vector<uint8_t> wlive(wcell.size(), 0);  // written so far (in program order)
    auto col_read = [&](uint32_t sec, uint32_t col, int32_t sh, std::string &e) -> int {
        const uint32_t j = col_slot(sec, col);
        if (is_written(j)) {
            auto it = wreg.find(std::make_pair(j, sh));
            if (it != wreg.end() && wlive[it->second]) {
                e = "w" + std::to_string(it->second) + "`";
                return 0;
            }
            if (sh != 0) return 1;  // cross-row read of a written column: interpreter
        }
        e.assign("C(", 2);
        app_num(e, j);
        e += ',';
        if (sh < 0) e += '-';
        app_num(e, (uint64_t)(sh < 0 ? -(int64_t)sh : sh));
        e += ",i`)";
        return 0;
    };
    auto kconst = [&](const uint64_t *v, int dim) {
        const size_t o = kc.size();
        for (int t = 0; t < dim; t++) kc.push_back(v[t] % 0xFFFFFFFF00000001ULL);
        return o;
    };
    bool uses_x = false;
    auto operand = [&](uint32_t idx, Expr &x) -> int {
        const zxp_operand &o = in.opnd[idx];
        char b[160];
        switch (o.kind) {
        case ZXP_TMP1: x = {"a" + std::to_string(idx) + "`", 1}; return 0;
        case ZXP_TMP3: x = {"b" + std::to_string(idx) + "`", 3}; return 0;
        case ZXP_COL: x.dim = 1; return col_read(o.a, o.b, (int32_t)o.c, x.e);
        case ZXP_COL3: {
            std::string c0, c1, c2;
            if (col_read(o.a, o.b, (int32_t)o.c, c0) || col_read(o.a, o.b + 1, (int32_t)o.c, c1) ||
                col_read(o.a, o.b + 2, (int32_t)o.c, c2))
                return 1;
            x = {"gl3{{" + c0 + "," + c1 + "," + c2 + "}}", 3};
            return 0;
        }
        case ZXP_LIT: {
            const uint64_t v = ((uint64_t)o.a | ((uint64_t)o.b << 32)) % 0xFFFFFFFF00000001ULL;
            snprintf(b, sizeof(b), "0x%llxULL", (unsigned long long)v);
            x = {b, 1};
            return 0;
        }
        case ZXP_PUB:
        case ZXP_CHAL:
        case ZXP_EVAL:
        case ZXP_IMM: {
            const uint64_t *v = o.kind == ZXP_PUB    ? in.publics + o.a
                                : o.kind == ZXP_CHAL ? in.challenges + 3 * o.a
                                : o.kind == ZXP_EVAL ? in.evals + 3 * o.a
                                                     : in.csts + 3 * o.a;
            const int dim = o.kind == ZXP_PUB ? 1 : o.kind == ZXP_IMM ? (int)o.b : 3;
            const size_t off = kconst(v, dim);
            if (dim == 1)
                snprintf(b, sizeof(b), "p.kc[%zu]", off);
            else
                snprintf(b, sizeof(b), "gl3{{p.kc[%zu],p.kc[%zu],p.kc[%zu]}}", off, off + 1, off + 2);
            x = {b, dim};
            return 0;
        }
        case ZXP_X: uses_x = true; x = {"xv`", 1}; return 0;
        case ZXP_XDIV: x = {"gl3{{gload(p.xdiv+3*i`),gload(p.xdiv+3*i`+1),gload(p.xdiv+3*i`+2)}}", 3}; return 0;
        case ZXP_XDIVW: x = {"gl3{{gload(p.xdivw+3*i`),gload(p.xdivw+3*i`+1),gload(p.xdivw+3*i`+2)}}", 3}; return 0;
        case ZXP_ZI: x = {"gload(p.zh + (i` & p.zmask))", 1}; return 0;
        default: return 1;
        }
    };
    // limb table layout: Dot3 inits 3 words in 4-word slots, terms 6 words in
    // 8-word slots, so the kernel reads them with 16-byte vector loads
    auto align_kl = [&](size_t a) {
        while (kl.size() % a) kl.push_back(0);
    };
    auto limbs3 = [&](uint64_t c) {  // Dot3 constant init: 22/21/21-bit limbs of c
        kl.push_back((uint32_t)(c & ((1u << 22) - 1)));
        kl.push_back((uint32_t)((c >> 22) & ((1u << 21) - 1)));
        kl.push_back((uint32_t)(c >> 43));
        kl.push_back(0);
    };
    auto limbs6x3 = [&](const uint64_t coef[3]) {  // term limbs of the three components; returns the slot
        align_kl(8);
        const size_t kt = kl.size();
        for (int j = 0; j < 3; j++) {
            uint32_t l6[6];
            zxp_limbs6(coef[j] % 0xFFFFFFFF00000001ULL, l6);
            kl.insert(kl.end(), l6, l6 + 6);
            kl.push_back(0);
            kl.push_back(0);
        }
        return kt;
    };
    std::string body;
    // assignment of a value expression to a destination operand
    auto assign = [&](uint32_t didx, const Expr &r) -> int {
        const zxp_operand &d = in.opnd[didx];
        if ((d.kind == ZXP_COL || d.kind == ZXP_COL3) && d.a != ZXP_SEC_SCRATCH && store_now(d.a, d.b)) {
            // a column the program never reads: stored here, on row (i + shift) & m
            const uint32_t nc = d.kind == ZXP_COL3 ? 3 : 1;
            for (uint32_t c = 1; c < nc; c++)
                if (!store_now(d.a, d.b + c)) return 1;  // mixed triple: keep the deferred form simple
            const int32_t sh = (int32_t)d.c;
            if (d.kind == ZXP_COL)
                appendf(body, "ZK_STS(%u, %s%s, i`, %d);\n", col_slot(d.a, d.b), r.e.c_str(), r.dim == 3 ? ".v[0]" : "",
                        sh);
            else if (r.dim == 3)
                appendf(body, "{ const gl3 t_ = %s; ZK_STS(%u, t_.v[0], i`, %d); ZK_STS(%u, t_.v[1], i`, %d); "
                              "ZK_STS(%u, t_.v[2], i`, %d); }\n",
                        r.e.c_str(), col_slot(d.a, d.b), sh, col_slot(d.a, d.b + 1), sh, col_slot(d.a, d.b + 2), sh);
            else
                appendf(body, "ZK_STS(%u, %s, i`, %d); ZK_STS(%u, 0, i`, %d); ZK_STS(%u, 0, i`, %d);\n",
                        col_slot(d.a, d.b), r.e.c_str(), sh, col_slot(d.a, d.b + 1), sh, col_slot(d.a, d.b + 2), sh);
            return 0;
        }
        if ((d.kind == ZXP_COL || d.kind == ZXP_COL3) && d.a == ZXP_SEC_SCRATCH) {  // carried value: stored at once
            if (d.c != 0) return 1;
            if (d.kind == ZXP_COL)
                appendf(body, "ZK_ST(%u, %s%s, i`);\n", col_slot(d.a, d.b), r.e.c_str(), r.dim == 3 ? ".v[0]" : "");
            else if (r.dim == 3)
                appendf(body, "{ const gl3 t_ = %s; ZK_ST(%u, t_.v[0], i`); ZK_ST(%u, t_.v[1], i`); ZK_ST(%u, t_.v[2], i`); }\n",
                        r.e.c_str(), col_slot(d.a, d.b), col_slot(d.a, d.b + 1), col_slot(d.a, d.b + 2));
            else
                appendf(body, "ZK_ST(%u, %s, i`); ZK_ST(%u, 0, i`); ZK_ST(%u, 0, i`);\n", col_slot(d.a, d.b), r.e.c_str(),
                        col_slot(d.a, d.b + 1), col_slot(d.a, d.b + 2));
            return 0;
        }
        switch (d.kind) {
        case ZXP_TMP1:
            body += 'a';
            app_num(body, didx);
            body += "` = ";
            body += r.e;
            if (r.dim == 3) body += ".v[0]";
            body += ";\n";
            return 0;
        case ZXP_TMP3:
            if (r.dim == 3) {
                body += 'b';
                app_num(body, didx);
                body += "` = ";
                body += r.e;
                body += ";\n";
            }
            else
                appendf(body, "b%u` = gl3{{%s, 0, 0}};\n", didx, r.e.c_str());
            return 0;
        case ZXP_COL: {
            const uint32_t j = wreg.at(std::make_pair(col_slot(d.a, d.b), (int32_t)d.c));
            appendf(body, "w%u` = %s%s;\n", j, r.e.c_str(), r.dim == 3 ? ".v[0]" : "");
            wlive[j] = 1;
            return 0;
        }
        case ZXP_COL3: {
            uint32_t j[3];
            for (int c = 0; c < 3; c++) j[c] = wreg.at(std::make_pair(col_slot(d.a, d.b + c), (int32_t)d.c));
            if (r.dim == 3)
                appendf(body, "{ const gl3 t_ = %s; w%u` = t_.v[0]; w%u` = t_.v[1]; w%u` = t_.v[2]; }\n", r.e.c_str(),
                        j[0], j[1], j[2]);
            else
                appendf(body, "w%u` = %s; w%u` = 0; w%u` = 0;\n", j[0], r.e.c_str(), j[1], j[2]);
            for (int c = 0; c < 3; c++) wlive[j[c]] = 1;
            return 0;
        }
        default: return 1;
        }
    };
    // DOT plan.  A term whose source is a temporary is accumulated right where
    // that temporary is defined (exact integer sums commute), so temporaries
    // feeding a linear combination die at once instead of staying live until
    // the DOT: register pressure stays that of one constraint at a time.
    struct Stream {
        uint32_t dot;
        bool three;
        std::string val;
        size_t kt;
    };
    std::vector<std::vector<Stream>> stream(in.n_instr);
    std::vector<uint8_t> streamed_term;  // per DOT term index: accumulated at the source's definition
    // Streaming a term opens the DOT's accumulators (3 or 9 words) at the
    // source's definition: for a source defined long before its DOT that
    // holds more registers than keeping the source (1 or 3 words) -- the
    // fork-9 step42ns peaked at ~1,300 live words with unbounded streaming
    // against ~110 without.  Only sources defined at most STREAM_SPAN
    // instructions before their DOT are streamed.
    // Small programs (< 1,000 compiled instructions: one or two Horner
    // accumulators over the whole program) stream without limit.
    const int64_t stream_span = in.n_instr < 1000 ? INT64_MAX / 4 : 24;
    {
        uint32_t nt = 0;
        for (uint32_t k = 0; k < in.n_instr; k++)
            if (in.ins[k].op == ZXP_DOT1 || in.ins[k].op == ZXP_DOT3) nt = std::max(nt, in.ins[k].a + in.ins[k].b);
        streamed_term.assign(nt, 0);
    }
    // Large programs (block-split, below) choose per DOT where to open its
    // accumulators by a register cost
    const bool cost_stream = in.n_instr >= 1000 || in.force_split;
    std::vector<int64_t> last_read(in.n_opnd ? in.n_opnd : 1, -1);  // per SSA operand
    for (uint32_t k = 0; k < in.n_instr; k++) {
        const zxp_instr &I = in.ins[k];
        if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
            for (uint32_t t = I.a; t < I.a + I.b; t++)
                if (in.terms[t].src != ZXP_TERM_ONE && in.terms[t].src < last_read.size()) last_read[in.terms[t].src] = k;
        } else {
            if (I.a < last_read.size()) last_read[I.a] = k;
            if (I.op != ZXP_COPY && I.b < last_read.size()) last_read[I.b] = k;
        }
    }
    // Only programs of 1000 compiled instructions or more are split: the
    // opaque branch costs registers (config-4 FRI polynomial: 74 -> 200
    // VGPRs, 9 -> 57 ms), and small programs compile in seconds as one block.
    const bool split = in.n_instr >= 1000 || in.force_split;
    // ---- fused column chains (the FRI polynomial, step52ns) -------------
    // A Horner chain over committed columns compiles to a chain of DOTs of at
    // most max_terms terms, each carrying the previous one as an F_p^3 term;
    // the FRI polynomial has one chain per opening point and most columns sit
    // in several of them (zkEVM-shaped step52ns: 3 chains, 3,778 column terms
    // over 1,497 columns; config-4: 397 over 189), each read again from HBM
    // at a distance no cache holds.  A non-split program evaluates up to
    // FUSE_MAX such chains together where the first link stood: each chain is
    // unrolled on the host (a link's column coefficient mapped through the
    // later links' carry maps, exact arithmetic mod p), the columns are
    // grouped by the set of chains they appear in, and each group is one loop
    // that reads a column once and accumulates it into all of its chains.
    // Same values (the chain sum is linear; accumulators are reduced every
    // FUSE_PIECE columns).  Measured (A/B on one box): zkEVM-shaped FRI
    // polynomial at 2^23 rows 69.4 -> 38.4 ms with 4 column loads in flight
    // per iteration, 33.5 ms with 8 (FUSE_U); the config-4 one
    // (397 column terms) 9.3 -> 10.4 ms with 4, 8.1 ms with 8.  Small chains
    // inside other programs (config-4 quotient, step3prev: 20-24 columns)
    // ran slower fused, so a program is fused only when its chains hold at
    // least half of its column terms and fuse_min (128) or more -- the FRI
    // polynomials.
    constexpr int FUSE_MAX = 4;
    constexpr uint32_t FUSE_PIECE = 224;
    constexpr size_t fuse_min = 128;
    constexpr size_t fuse_u = 8;  // column loads in flight per fused-loop iteration
    std::vector<int32_t> fused(in.n_instr, -1);  // chain of a fused link
    std::vector<std::vector<uint32_t>> fchains;   // links in order, per fused chain
    uint32_t fuse_at = UINT32_MAX;                // where the fused chains are evaluated
    if (!split) {
        // a link: DOT3 whose terms are column reads (columns the program never
        // writes), constants, and the whole previous link (its only reader)
        std::map<uint32_t, uint32_t> def_at;  // SSA operand -> defining instruction
        for (uint32_t k = 0; k < in.n_instr; k++) def_at[in.ins[k].dst] = k;
        std::vector<int64_t> prev(in.n_instr, -2);  // -2 not a link, -1 first link, else previous link
        std::vector<uint32_t> readers(in.n_opnd ? in.n_opnd : 1, 0);
        for (uint32_t k = 0; k < in.n_instr; k++) {
            const zxp_instr &I = in.ins[k];
            if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
                std::set<uint32_t> srcs;
                for (uint32_t t = I.a; t < I.a + I.b; t++)
                    if (in.terms[t].src != ZXP_TERM_ONE && in.terms[t].src < in.n_opnd) srcs.insert(in.terms[t].src);
                for (uint32_t x : srcs) readers[x]++;
            } else {
                if (I.a < in.n_opnd) readers[I.a]++;
                if (I.op != ZXP_COPY && I.b < in.n_opnd && I.b != I.a) readers[I.b]++;
            }
        }
        for (uint32_t k = 0; k < in.n_instr; k++) {
            const zxp_instr &I = in.ins[k];
            if (I.op != ZXP_DOT3 || in.opnd[I.dst].kind != ZXP_TMP3) continue;
            int64_t pv = -1;
            bool ok = true;
            uint32_t ncol = 0;
            for (uint32_t t = I.a; t < I.a + I.b && ok; t++) {
                const zxp_term &tm = in.terms[t];
                if (tm.src == ZXP_TERM_ONE) continue;
                const zxp_operand &o = in.opnd[tm.src];
                if (o.kind == ZXP_COL) {
                    ok = !is_written(col_slot(o.a, o.b));
                    ncol++;
                } else if (o.kind == ZXP_TMP3 && def_at.count(tm.src) && prev[def_at[tm.src]] != -2 &&
                           readers[tm.src] == 1 && (pv < 0 || pv == (int64_t)def_at[tm.src])) {
                    pv = def_at[tm.src];
                } else {
                    ok = false;
                }
            }
            if (ok && (ncol > 0 || pv >= 0)) prev[k] = pv;
        }
        // chains: from links nobody continues, walk back
        std::vector<uint8_t> continued(in.n_instr, 0);
        for (uint32_t k = 0; k < in.n_instr; k++)
            if (prev[k] >= 0) continued[prev[k]] = 1;
        std::vector<std::vector<uint32_t>> cand;
        for (uint32_t k = 0; k < in.n_instr; k++) {
            if (prev[k] == -2 || continued[k]) continue;
            std::vector<uint32_t> ch;
            for (int64_t x = k; x >= 0; x = prev[x]) ch.push_back((uint32_t)x);
            std::reverse(ch.begin(), ch.end());
            cand.push_back(ch);
        }
        // the largest chains (by column terms), if at least two share columns
        auto ncols_of = [&](const std::vector<uint32_t> &ch) {
            size_t n = 0;
            for (uint32_t x : ch) n += in.ins[x].b;
            return n;
        };
        std::stable_sort(cand.begin(), cand.end(),
                         [&](const std::vector<uint32_t> &a, const std::vector<uint32_t> &b) { return ncols_of(a) > ncols_of(b); });
        if (cand.size() > (size_t)FUSE_MAX) cand.resize(FUSE_MAX);
        std::map<std::pair<uint32_t, int32_t>, uint32_t> in_chains;  // (slot, shift) -> chain mask
        for (size_t g = 0; g < cand.size(); g++)
            for (uint32_t x : cand[g])
                for (uint32_t t = in.ins[x].a; t < in.ins[x].a + in.ins[x].b; t++) {
                    const zxp_term &tm = in.terms[t];
                    if (tm.src == ZXP_TERM_ONE || in.opnd[tm.src].kind != ZXP_COL) continue;
                    const zxp_operand &o = in.opnd[tm.src];
                    in_chains[{col_slot(o.a, o.b), (int32_t)o.c}] |= 1u << g;
                }
        size_t shared = 0, terms = 0, all_terms = 0;
        for (auto &kv : in_chains) {
            shared += __builtin_popcount(kv.second) > 1;
            terms += __builtin_popcount(kv.second);
        }
        for (uint32_t k = 0; k < in.n_instr; k++)  // the program's column terms
            if (in.ins[k].op == ZXP_DOT1 || in.ins[k].op == ZXP_DOT3)
                for (uint32_t t = in.ins[k].a; t < in.ins[k].a + in.ins[k].b; t++)
                    all_terms += in.terms[t].src != ZXP_TERM_ONE && in.opnd[in.terms[t].src].kind == ZXP_COL;
        if (cand.size() >= 2 && shared > 0 && terms >= fuse_min && 2 * terms >= all_terms) {
            fchains = cand;
            for (size_t g = 0; g < fchains.size(); g++)
                for (uint32_t x : fchains[g]) {
                    fused[x] = (int32_t)g;
                    fuse_at = std::min(fuse_at, x);
                }
        }
    }
    // unrolled chains: per chain, the coefficient (F_p^3) of every column and
    // the constant, mapped through the later links' carry maps
    struct FusedCol {
        uint32_t slot;
        int32_t sh;
        uint32_t mask;  // chains the column appears in (structure, not values)
        uint64_t c[FUSE_MAX][3];
    };
    std::vector<FusedCol> fcols;  // in order of first appearance
    std::vector<std::array<uint64_t, 3>> fconst(fchains.size(), std::array<uint64_t, 3>{0, 0, 0});
    if (!fchains.empty()) {
        constexpr uint64_t P = 0xFFFFFFFF00000001ULL;
        auto fadd = [](uint64_t a, uint64_t b) {
            const uint64_t s = a + b;
            return (s < a || s >= P) ? s - P : s;
        };
        auto fmul = [](uint64_t a, uint64_t b) { return h_mul(a, b); };
        std::map<std::pair<uint32_t, int32_t>, size_t> fidx;
        for (size_t g = 0; g < fchains.size(); g++)
            for (uint32_t x : fchains[g])
                for (uint32_t t = in.ins[x].a; t < in.ins[x].a + in.ins[x].b; t++) {
                    const zxp_term &tm = in.terms[t];
                    if (tm.src == ZXP_TERM_ONE || in.opnd[tm.src].kind != ZXP_COL) continue;
                    const zxp_operand &o = in.opnd[tm.src];
                    const std::pair<uint32_t, int32_t> key{col_slot(o.a, o.b), (int32_t)o.c};
                    if (!fidx.count(key)) {
                        fidx[key] = fcols.size();
                        FusedCol fc;
                        memset(&fc, 0, sizeof(fc));
                        fc.slot = key.first;
                        fc.sh = key.second;
                        fcols.push_back(fc);
                    }
                }
        for (size_t g = 0; g < fchains.size(); g++) {
            // M: the map from a link's value to the chain's final value (3x3 over F_p)
            uint64_t M[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
            for (size_t li = fchains[g].size(); li-- > 0;) {
                const zxp_instr &I = in.ins[fchains[g][li]];
                uint64_t L[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};  // previous link -> this link
                for (uint32_t t = I.a; t < I.a + I.b; t++) {
                    const zxp_term &tm = in.terms[t];
                    uint64_t a[3], v[3];
                    for (int j = 0; j < 3; j++) a[j] = tm.coef[j] % P;
                    for (int r = 0; r < 3; r++) {
                        v[r] = 0;
                        for (int j = 0; j < 3; j++) v[r] = fadd(v[r], fmul(M[r][j], a[j]));
                    }
                    if (tm.src == ZXP_TERM_ONE) {
                        for (int r = 0; r < 3; r++) fconst[g][r] = fadd(fconst[g][r], v[r]);
                    } else if (in.opnd[tm.src].kind == ZXP_COL) {
                        const zxp_operand &o = in.opnd[tm.src];
                        FusedCol &fc = fcols[fidx[{col_slot(o.a, o.b), (int32_t)o.c}]];
                        fc.mask |= 1u << g;
                        for (int r = 0; r < 3; r++) fc.c[g][r] = fadd(fc.c[g][r], v[r]);
                    } else {  // the previous link, component tm.comp
                        for (int r = 0; r < 3; r++) L[r][tm.comp] = fadd(L[r][tm.comp], a[r]);
                    }
                }
                uint64_t M2[3][3];
                for (int r = 0; r < 3; r++)
                    for (int c = 0; c < 3; c++) {
                        M2[r][c] = 0;
                        for (int j = 0; j < 3; j++) M2[r][c] = fadd(M2[r][c], fmul(M[r][j], L[j][c]));
                    }
                memcpy(M, M2, sizeof(M));
            }
        }
    }
    std::vector<size_t> dot_k0(in.n_instr, 0);
    std::vector<uint32_t> first_use(in.n_instr, UINT32_MAX);  // declaration point of DOT k's accumulators
    {
        std::vector<int64_t> last1(in.n_tmp1 + 1, -1), last3(in.n_tmp3 + 1, -1);
        for (uint32_t k = 0; k < in.n_instr; k++) {
            const zxp_instr &I = in.ins[k];
            if (fused[k] >= 0) {  // evaluated with its chain at fuse_at
                const zxp_operand &D = in.opnd[I.dst];
                if (D.kind == ZXP_TMP3) last3[D.a] = (k == fchains[fused[k]].back()) ? (int64_t)fuse_at : (int64_t)k;
                continue;
            }
            if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
                const bool three = I.op == ZXP_DOT3;
                uint64_t c0[3] = {0, 0, 0};
                for (uint32_t t = I.a; t < I.a + I.b; t++)
                    if (in.terms[t].src == ZXP_TERM_ONE)
                        for (int j = 0; j < 3; j++) {
                            const uint64_t P = 0xFFFFFFFF00000001ULL, v = in.terms[t].coef[j] % P;
                            const uint64_t sum = c0[j] + v;
                            c0[j] = (sum < v || sum >= P) ? sum - P : sum;
                        }
                align_kl(4);
                dot_k0[k] = kl.size();
                for (int j = 0; j < 3; j++) limbs3(c0[j]);
                first_use[k] = k;
                // cost mode: open the accumulators (A VGPRs) at the definition
                // d_j that minimises A (k - d_j) + sum over the earlier-defined
                // sources w_i (k - d_i) (those wait in registers); only sources
                // whose last read is this DOT count (others stay live anyway)
                int64_t d_open = INT64_MIN;
                if (cost_stream) {
                    std::vector<std::pair<int64_t, int64_t>> cand;  // (definition, VGPRs freed)
                    for (uint32_t t = I.a; t < I.a + I.b; t++) {
                        const zxp_term &tm = in.terms[t];
                        if (tm.src == ZXP_TERM_ONE) continue;
                        const zxp_operand &o = in.opnd[tm.src];
                        if (o.kind != ZXP_TMP1 && o.kind != ZXP_TMP3) continue;
                        const int64_t d = o.kind == ZXP_TMP1 ? last1[o.a] : last3[o.a];
                        if (d < 0 || last_read[tm.src] != (int64_t)k) continue;
                        cand.push_back({d, 2});  // per term: a base value or one component of an F_p^3 temporary
                    }
                    std::sort(cand.begin(), cand.end());
                    const int64_t A = three ? 18 : 6;
                    int64_t wait = 0;  // sum w_i (k - d_i) over the sources before j
                    for (const auto &c : cand) wait += c.second * ((int64_t)k - c.first);
                    int64_t best = wait;  // no streaming
                    int64_t acc = 0;
                    for (size_t j = 0; j < cand.size(); j++) {
                        const int64_t c = A * ((int64_t)k - cand[j].first) + acc;
                        if (c < best) {
                            best = c;
                            d_open = cand[j].first;
                        }
                        acc += cand[j].second * ((int64_t)k - cand[j].first);
                    }
                    if (d_open == INT64_MIN) d_open = INT64_MAX;
                }
                for (uint32_t t = I.a; t < I.a + I.b; t++) {
                    const zxp_term &tm = in.terms[t];
                    if (tm.src == ZXP_TERM_ONE) continue;
                    const zxp_operand &o = in.opnd[tm.src];
                    if (o.kind != ZXP_TMP1 && o.kind != ZXP_TMP3) continue;
                    const int64_t d = o.kind == ZXP_TMP1 ? last1[o.a] : last3[o.a];
                    if (d < 0) continue;  // never written: the value is 0
                    if (cost_stream ? (d < d_open || last_read[tm.src] != (int64_t)k) : (int64_t)k - d > stream_span)
                        continue;  // read at the DOT instead
                    streamed_term[t] = 1;
                    Stream st;
                    st.dot = k;
                    st.three = three;
                    st.val = o.kind == ZXP_TMP1 ? "a" + std::to_string(tm.src) + "`"
                                                : "b" + std::to_string(tm.src) + "`.v[" + std::to_string(tm.comp) + "]";
                    st.kt = limbs6x3(tm.coef);
                    stream[d].push_back(st);
                    first_use[k] = std::min<uint32_t>(first_use[k], (uint32_t)d);
                }
            }
            const zxp_operand &D = in.opnd[I.dst];
            if (D.kind == ZXP_TMP1) last1[D.a] = k;
            if (D.kind == ZXP_TMP3) last3[D.a] = k;
        }
    }
    std::vector<std::vector<uint32_t>> declare_at(in.n_instr);
    for (uint32_t k = 0; k < in.n_instr; k++)
        if (first_use[k] != UINT32_MAX) declare_at[first_use[k]].push_back(k);
    // Compile time: LLVM's instruction selection and machine scheduler are
    // superlinear in basic-block size (a 600-instruction program took ~60 s
    // as one block).  Every `block` (1 KB) of source the body opens a
    // new block behind a uniform branch on an opaque 1 (zk_one(): an
    // s_mov_b32 the optimiser cannot see through, so it cannot merge the
    // blocks back), so each block is compiled on its own.  The block size also
    // bounds how far the scheduler hoists column loads: quarter-size
    // step42ns-shaped program at 2^24 rows, 256 / 512 / 1024 / 4096 bytes ->
    // 184 / 246 / 246 / 512+spills VGPRs, 453 / 359 / 303 / 394 ms, hiprtc
    // 63 / 56 / 80 / 116 s.
    // source bytes per block (segments: 512, round 6 -- paired with the
    // prefetch: without it the 512-byte segments ran 8 % slower)
    const size_t block = in.force_split ? (seg_ab().block ? seg_ab().block : 512) : 1024;
    // Limb chunks in LDS: a split program whose limb
    // table is too large for LDS reads it from global memory, one wave-uniform
    // 16 + 8-byte vector load pair per term, each taking the texture
    // addresser's full 64-lane path.  In this mode the table is rewritten in
    // emission order (kmap), every code block's limbs form one contiguous
    // chunk of <= JIT_KCHUNK words, the workgroup copies the next block's
    // chunk into the other half of an LDS double buffer (one 16-byte load per
    // thread, issued at the block's start) and a barrier closes each block.
    // Quarter-size step42ns-shaped program at 2^24 rows: 251 -> 189 ms
    // (global vector loads of the limbs 25 K -> 6.7 K per wave).  Every split
    // program.
    const bool kchunk = split;
    std::vector<uint32_t> kl2;
    size_t blk_lo = 0, blk_no = 0;
    auto kmap = [&](size_t off, size_t n) -> size_t {  // n words of kl at off, in emission order
        if (!kchunk) return off;
        const size_t o = kl2.size();
        kl2.insert(kl2.end(), kl.begin() + off, kl.begin() + off + n);
        while (kl2.size() % 4) kl2.push_back(0);
        return o;
    };
    // DOT accumulators are declared at function scope (the body is split into
    // blocks, below) and initialised where the first term arrives
    std::string dot_decls;
    auto emit_declarations = [&](uint32_t at) {
        for (uint32_t k : declare_at[at]) {
            const size_t k0 = dot_k0[k];
            if (in.ins[k].op == ZXP_DOT3) {
                appendf(dot_decls, "Dot3 D%u_0`, D%u_1`, D%u_2`;\n", k, k, k);
                const size_t m0 = kmap(k0, 12);
                appendf(body, "D%u_0` = Dot3(K + %zu); D%u_1` = Dot3(K + %zu); D%u_2` = Dot3(K + %zu);\n", k, m0, k,
                        m0 + 4, k, m0 + 8);
            } else {
                appendf(dot_decls, "Dot3 D%u_0`;\n", k);
                appendf(body, "D%u_0` = Dot3(K + %zu);\n", k, kmap(k0, 4));
            }
        }
    };
    // A limb chunk spans as many code blocks as its limbs fill (a workgroup
    // barrier every ~3-4 blocks; a chunk and barrier per block, the round-3
    // form, measured 43.3 against 45.4 Mrow/s on the zkEVM-sized quotient)
    size_t block_start = 0;
    auto chunk_head = [&] {  // LDS base of this chunk; the next chunk's start patched in at the end
        appendf(body, "const uint32_t *K = kbuf + %d - %zu; pf_ = kpre(p.kl, @KLO%zu@);\n",
                (int)(blk_no & 1) * JIT_KCHUNK, blk_lo, blk_no + 1);
    };
    std::vector<size_t> klo_of;  // chunk start of chunk b
    auto maybe_split = [&] {
        const bool full = kchunk && kl2.size() - blk_lo > JIT_KCHUNK - 256;
        if (split && (body.size() - block_start >= block || full)) {
            if (full) {
                appendf(body, "kput(kbuf + %d, pf_);\n}\n__syncthreads();\n", (int)((blk_no + 1) & 1) * JIT_KCHUNK);
                blk_lo = kl2.size();
                blk_no++;
                klo_of.push_back(blk_lo);
                body += "if (zk_one()) {\n";
                chunk_head();
            } else if (kchunk) {  // same chunk, new code block
                appendf(body, "}\nif (zk_one()) {\nconst uint32_t *K = kbuf + %d - %zu;\n", (int)(blk_no & 1) * JIT_KCHUNK,
                        blk_lo);
            } else {
                body += "}\nif (zk_one()) { ZK_KREFRESH\n";
            }
            block_start = body.size();
        }
    };
    body += split ? "if (zk_one()) {\n" : "{\n";
    if (kchunk) {
        klo_of.push_back(0);
        chunk_head();
    }
    auto emit_streams = [&](uint32_t at) {
        for (const Stream &st : stream[at]) {
            maybe_split();
            const size_t kt = kmap(st.kt, st.three ? 24 : 8);
            app_term(body, st.val, st.dot, kt, st.three);
        }
    };
    // the fused chains (above), where their first link stood
    auto emit_fused = [&]() -> int {
        const size_t G = fchains.size();
        body += "{\n";
        for (size_t g = 0; g < G; g++) {
            align_kl(4);
            const size_t o = kl.size();
            for (int j = 0; j < 3; j++) limbs3(fconst[g][j]);
            appendf(body, "Dot3 F%zu_0` = Dot3(K + %zu), F%zu_1` = Dot3(K + %zu), F%zu_2` = Dot3(K + %zu);\n", g, o, g, o + 4,
                    g, o + 8);
        }
        std::vector<uint32_t> fill(G, 0);  // terms since the chain's last reduction
        for (uint32_t mask = 1; mask < (1u << G); mask++) {
            std::vector<const FusedCol *> cols;
            for (const FusedCol &fc : fcols)
                if (fc.mask == mask) cols.push_back(&fc);
            if (cols.empty()) continue;
            std::vector<int> mem;
            for (size_t g = 0; g < G; g++)
                if (mask >> g & 1) mem.push_back((int)g);
            const size_t R = mem.size();
            for (size_t p0 = 0; p0 < cols.size(); p0 += FUSE_PIECE) {
                const size_t n = std::min<size_t>(FUSE_PIECE, cols.size() - p0);
                const size_t np = (n + fuse_u - 1) / fuse_u * fuse_u;
                const size_t off = zt.size();
                for (size_t e = 0; e < np; e++) {
                    const FusedCol &fc = *cols[p0 + std::min(e, n - 1)];
                    for (size_t r = 0; r < R; r++) {
                        JitTerm jt;
                        memset(&jt, 0, sizeof(jt));
                        jt.ptr = cp[fc.slot];
                        jt.sh = fc.sh;
                        if (e < n)  // padding entries: zero limbs
                            for (int j = 0; j < 3; j++) zxp_limbs6(fc.c[mem[r]][j] % 0xFFFFFFFF00000001ULL, jt.c[j]);
                        zt.push_back(jt);
                    }
                }
                for (int g : mem)
                    if (fill[g] + np > 240) {  // Dot3 accumulators: reduce before 2^63 (gl_device.hpp)
                        appendf(body, "{ const uint64_t x0_ = F%d_0`.fin(), x1_ = F%d_1`.fin(), x2_ = F%d_2`.fin(); "
                                      "F%d_0` = Dot3(); F%d_0`.lane(x0_); F%d_1` = Dot3(); F%d_1`.lane(x1_); "
                                      "F%d_2` = Dot3(); F%d_2`.lane(x2_); }\n",
                                g, g, g, g, g, g, g, g, g);
                        fill[g] = 1;
                    }
                for (int g : mem) fill[g] += (uint32_t)np;
                appendf(body, "for (int q_ = 0; q_ < %zu; q_ += %zu) {\nconst JitTerm *t_ = ZT + %zu + (size_t)q_ * %zu;\n"
                              "uint64_t fv`[%zu];\n", np, fuse_u, off, R, fuse_u);
                appendf(body, "_Pragma(\"unroll\") for (int u_ = 0; u_ < %zu; u_++) fv`[u_] = gload(t_[u_ * %zu].ptr + "
                              "((i` + (uint64_t)t_[u_ * %zu].sh) & m));\n", fuse_u, R, R);
                appendf(body, "_Pragma(\"unroll\") for (int u_ = 0; u_ < %zu; u_++) {\n", fuse_u);
                for (size_t r = 0; r < R; r++)
                    appendf(body, "F%d_0`.term(fv`[u_], t_[u_ * %zu + %zu].c[0]); F%d_1`.term(fv`[u_], t_[u_ * %zu + %zu].c[1]); "
                                  "F%d_2`.term(fv`[u_], t_[u_ * %zu + %zu].c[2]);\n",
                            mem[r], R, r, mem[r], R, r, mem[r], R, r);
                body += "}\n}\n";
            }
        }
        for (size_t g = 0; g < G; g++) {
            char fin[128];
            snprintf(fin, sizeof(fin), "gl3{{F%zu_0`.fin(), F%zu_1`.fin(), F%zu_2`.fin()}}", g, g, g);
            if (assign(in.ins[fchains[g].back()].dst, Expr{fin, 3})) return 1;
        }
        body += "}\n";
        return 0;
    };
    for (uint32_t k = 0; k < in.n_instr; k++) {
        const zxp_instr &I = in.ins[k];
        maybe_split();
        emit_declarations(k);
        if (fused[k] >= 0) {
            if (k == fuse_at) {
                if (emit_fused()) return 1;
                emit_streams(k);
            }
            continue;
        }
        if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
            const bool three = I.op == ZXP_DOT3;
            // column terms read from memory: looped from the term table when
            // there are many (code size, compile time), unrolled otherwise
            auto memcol = [&](const zxp_term &tm) {
                if (tm.src == ZXP_TERM_ONE) return false;
                const zxp_operand &o = in.opnd[tm.src];
                if (o.kind != ZXP_COL) return false;
                auto it = wreg.find(std::make_pair(col_slot(o.a, o.b), (int32_t)o.c));
                return !(it != wreg.end() && wlive[it->second]);
            };
            uint32_t n_mem = 0;
            for (uint32_t t = I.a; t < I.a + I.b; t++) n_mem += memcol(in.terms[t]);
            // (large programs unroll every term: a looped DOT reads its
            // term records through vector loads, one wait each, and holds its
            // accumulators and in-flight loads across the loop -- the
            // zkEVM-sized quotient 1.27 s with loops, 0.57 s without)
            const bool loop = !split && n_mem >= in.dot_loop_min;
            if (loop) {
                const size_t t0 = zt.size();
                for (uint32_t t = I.a; t < I.a + I.b; t++) {
                    const zxp_term &tm = in.terms[t];
                    if (!memcol(tm)) continue;
                    const zxp_operand &o = in.opnd[tm.src];
                    if (is_written(col_slot(o.a, o.b)) && o.c != 0) return 1;
                    JitTerm jt;
                    memset(&jt, 0, sizeof(jt));
                    jt.ptr = col_ptr(o.a, o.b);
                    jt.sh = (int64_t)(int32_t)o.c;
                    for (int j = 0; j < 3; j++) zxp_limbs6(tm.coef[j] % 0xFFFFFFFF00000001ULL, jt.c[j]);
                    zt.push_back(jt);
                }
                if (three)
                    appendf(body, "dot_cols<3>(D%u_0`, D%u_1`, D%u_2`, ZT + %zu, %u, i`, m);\n", k, k, k, t0, n_mem);
                else
                    appendf(body, "dot_cols<1>(D%u_0`, D%u_0`, D%u_0`, ZT + %zu, %u, i`, m);\n", k, k, k, t0, n_mem);
            }
            for (uint32_t t = I.a; t < I.a + I.b; t++) {
                const zxp_term &tm = in.terms[t];
                if (tm.src == ZXP_TERM_ONE) continue;
                const zxp_operand &o = in.opnd[tm.src];
                if (o.kind != ZXP_COL) {
                    if (o.kind != ZXP_TMP1 && o.kind != ZXP_TMP3) return 1;
                    if (streamed_term[t]) continue;  // accumulated at the temporary's definition
                    maybe_split();
                    const std::string v = o.kind == ZXP_TMP1
                                              ? "a" + std::to_string(tm.src) + "`"
                                              : "b" + std::to_string(tm.src) + "`.v[" + std::to_string(tm.comp) + "]";
                    const size_t kt = kmap(limbs6x3(tm.coef), three ? 24 : 8);
                    app_term(body, v, k, kt, three);
                    continue;
                }
                if (loop && memcol(tm)) continue;
                maybe_split();
                std::string e;
                if (col_read(o.a, o.b, (int32_t)o.c, e)) return 1;
                const size_t kt = kmap(limbs6x3(tm.coef), three ? 24 : 8);
                app_term(body, e, k, kt, three);
            }
            char fin[128];
            if (three)
                snprintf(fin, sizeof(fin), "gl3{{D%u_0`.fin(), D%u_1`.fin(), D%u_2`.fin()}}", k, k, k);
            else
                snprintf(fin, sizeof(fin), "D%u_0`.fin()", k);
            if (assign(I.dst, Expr{fin, three ? 3 : 1})) return 1;
            emit_streams(k);
            continue;
        }
        Expr A, B;
        if (operand(I.a, A)) return 1;
        if (I.op != ZXP_COPY && operand(I.b, B)) return 1;
        Expr R;
        const char *ea = A.e.c_str(), *eb = B.e.c_str();
        std::string s;
        if (I.op == ZXP_COPY) {
            R = A;
        } else if (I.op == ZXP_MUL) {
            if (A.dim == 3 && B.dim == 3)
                appendf(s, "gl3_mul(%s, %s)", ea, eb);
            else if (A.dim == 3)
                appendf(s, "gl3_mul1(%s, %s)", ea, eb);
            else if (B.dim == 3)
                appendf(s, "gl3_mul1(%s, %s)", eb, ea);
            else
                appendf(s, "gl_mul(%s, %s)", ea, eb);
            R = {s, std::max(A.dim, B.dim)};
        } else if (I.op == ZXP_ADD) {
            if (A.dim == 3 && B.dim == 3)
                appendf(s, "gl3_add(%s, %s)", ea, eb);
            else if (A.dim == 3)
                appendf(s, "gl3_add1(%s, %s)", ea, eb);
            else if (B.dim == 3)
                appendf(s, "gl3_add1(%s, %s)", eb, ea);
            else
                appendf(s, "gl_add(%s, %s)", ea, eb);
            R = {s, std::max(A.dim, B.dim)};
        } else if (I.op == ZXP_SUB) {
            if (A.dim == 3 && B.dim == 3)
                appendf(s, "gl3_sub(%s, %s)", ea, eb);
            else if (A.dim == 3)
                appendf(s, "gl3_sub1(%s, %s)", ea, eb);
            else if (B.dim == 3)
                appendf(s, "gl3_rsub1(%s, %s)", ea, eb);
            else
                appendf(s, "gl_sub(%s, %s)", ea, eb);
            R = {s, std::max(A.dim, B.dim)};
        } else {
            return 1;
        }
        if (assign(I.dst, R)) return 1;
        emit_streams(k);
    }
    if (kchunk) {  // chunk starts of the blocks' successors; the table in emission order, padded for the last copy
        klo_of.push_back(kl2.size());
        for (size_t b = 0; b + 1 < klo_of.size(); b++)
            if (klo_of[b + 1] - klo_of[b] > (size_t)JIT_KCHUNK)
                return 1;  // a block's limbs overflow the LDS chunk: unsupported shape, the interpreter runs it
        std::string b2;
        b2.reserve(body.size());
        size_t pos = 0;
        for (;;) {
            const size_t at = body.find("@KLO", pos);
            if (at == std::string::npos) break;
            const size_t end = body.find('@', at + 4);
            b2.append(body, pos, at - pos);
            const size_t b = strtoull(body.c_str() + at + 4, nullptr, 10);
            b2 += std::to_string(b < klo_of.size() ? klo_of[b] : kl2.size());
            pos = end + 1;
        }
        b2.append(body, pos, std::string::npos);
        body.swap(b2);
        kl2.resize(kl2.size() + JIT_KCHUNK, 0);
        kl.swap(kl2);
    }
    // assemble: prelude, params, declarations, body, deferred stores
    // Address space of the wave-uniform tables a kernel reads from global
    // memory (kas: the DOT limb table when not in LDS, cpas: the column
    // pointers; 0 generic = FLAT loads, 1 global = vector loads, 4 constant
    // = scalar loads).  Block-split
    // programs hide their limb table base behind an asm copy per block (so it
    // is not provably uniform and was read with FLAT loads, which also count
    // on LGKM_CNT) and loaded every column pointer with a vector load ahead of
    // the dependent column load: quarter-size step42ns-shaped program at 2^24
    // rows, limbs/pointers FLAT/vector 302 ms, global/vector 272, FLAT/scalar
    // 277, global/scalar 251 (default for split programs), scalar/scalar 293
    // (scalar limbs: 106 SGPRs, spills).  Small programs keep the compiler's
    // choice (their limbs already come from scalar loads).
    const int kas = split ? 1 : 0;
    const int cpas = split ? 4 : 0;
    src.clear();
    if ((kas == 1 || kas == 4) && !kchunk && !jit_kl_lds(kl.size()))
        appendf(src, "#define ZK_LIMB_AS __attribute__((address_space(%d)))\n", kas);
    if (cpas == 1 || cpas == 4) appendf(src, "#define ZK_CP_AS __attribute__((address_space(%d)))\n", cpas);
    // (field add / sub keep their second correction as a select: with the
    // wave-uniform branch of gl_device.hpp ZK_RB the branches split the long
    // straight-line blocks, zkEVM-shaped quotient 39.9 -> 32.8 Mrow/s)
    // DOT limb reads (gl_device.hpp Dot3::term_al): explicit 16 + 8-byte
    // loads for the split programs' LDS chunks (-O1), the struct copy the -O2
    // vectorizer merges for the others
    if (!kchunk) src += "#define ZK_LIMB_STRUCT 1\n";
    src += k_gl_device_src;
    appendf(src, "#define ZKJIT_KL_LDS %d\n", !kchunk && jit_kl_lds(kl.size()) ? 1 : 0);
    appendf(src, "#define ZKJIT_SPLIT %d\n", split ? 1 : 0);
    appendf(src, "#define ZKJIT_KL_CHUNK %d\n", kchunk ? JIT_KCHUNK : 0);  // large program: compile-time options (rtc_compile)
    // column terms per DOT-loop iteration (loads in flight; 8 / 16 measured neutral)
    src += "#define ZKJIT_UNROLL 4\n";
    if (in.waves_per_eu)
        appendf(src, "#define ZKJIT_WAVES __attribute__((amdgpu_waves_per_eu(%u)))\n", in.waves_per_eu);
    else
        src += "#define ZKJIT_WAVES\n";
    const uint32_t rows = jit_rows(split);
    appendf(src, "#define ZKJIT_ROWS %u\n", rows);
    // 32-bit column offsets from scalar bases (64-bit addresses, the round-3
    // form: 44.6 against 46.3 Mrow/s on the zkEVM-sized quotient)
    src += "#define ZKJIT_SADDR 1\n";
    uint32_t n_prefetch = 0;
    {
        // LDS column cache (lds_column_cache): block-split programs, 12
        // slots per lane and row (LDS: 2 KB per slot, row and workgroup; 16
        // slots measured +2 % on one box, -5 % on another)
        const SegAb &ab = seg_ab();
        const bool seg = split && in.force_split;  // a segment (zxp_segment)
        const uint32_t seg_w = in.waves_per_eu ? in.waves_per_eu : 4;
        const int lslots = seg ? (ab.waves ? (int)ab.slots : 16) : 12, lgap = 0;
        // LDS budget of one workgroup (64 KB): the limb double buffer (kbuf)
        // or the whole limb table, then as many cache slots as still fit
        // (none: the uncached source)
        const size_t lds_limbs = kchunk ? 2 * JIT_KCHUNK * 4 : (jit_kl_lds(kl.size()) ? kl.size() * 4 : 0);
        const size_t slot_bytes = (size_t)rows * 256 * 8;
        const size_t lds_budget = seg ? 160 * 1024 / seg_w : 64 * 1024;
        const int fit = lds_limbs >= lds_budget ? 0 : (int)((lds_budget - lds_limbs) / slot_bytes);
        const int slots = std::min(lslots, fit);
        const bool lc = split && slots > 0 && lds_column_cache(body, slots, lgap) > 0;
        appendf(src, "#define ZKJIT_LCACHE %d\n", lc ? slots : 0);
        n_prefetch = seg ? prefetch_blocks(body, ab.waves ? ab.prefetch : 16, ab.dist ? ab.dist : 1) : 0;
        if (n_prefetch) src += "#define CSV(v, s, r) zk_cs(zkc_ + ((s) * ZKJIT_ROWS + (r)) * 256, (v))\n";
    }
    src += k_kernel_head;
    // per-row text carries a ` (-> _r) and ~ (-> r) on its line; expand()
    // writes such a line once per row
    std::string decl = "const uint64_t i` = ib_ + ~ * S_;\n", tail;
    // Temporaries are named by SSA value (operand index), not by slot: the
    // code blocks sit behind branches the compiler cannot resolve, so a slot
    // variable reused through the program would keep every dead value it
    // held alive up to the slot's last read (the not-taken paths), i.e. all
    // slots live everywhere (~250 VGPRs on the zkEVM-sized quotient)
    {
        std::vector<uint8_t> seen(in.n_opnd, 0);
        for (uint32_t k = 0; k < in.n_instr; k++) {
            const uint32_t d = in.ins[k].dst;
            if (d >= in.n_opnd || seen[d]) continue;
            seen[d] = 1;
            if (in.opnd[d].kind == ZXP_TMP1 || in.opnd[d].kind == ZXP_TMP3) {
                decl += in.opnd[d].kind == ZXP_TMP1 ? "uint64_t a" : "gl3 b";
                app_num(decl, d);
                decl += "`;\n";
            }
        }
    }
    for (uint32_t r = 0; r < wcell.size(); r++) appendf(decl, "uint64_t w%u` = 0;\n", r);
    for (uint32_t r = 0; r < n_prefetch; r++) appendf(decl, "uint64_t zpf%u`;\n", r);
    if (uses_x)
        appendf(decl, "const uint64_t ex_` = i` << (%u - p.logomega);\n"
                     "const uint64_t xv` = gl_mul(p.x_start, gl_mul(gload(p.tw_lo + (ex_` & %lluULL)), gload(p.tw_hi + (ex_` >> %u))));\n",
                TW_MAX_LOG, (unsigned long long)(TW_LEVEL_SIZE - 1), TW_LEVEL_BITS);
    for (uint32_t r = 0; r < wcell.size(); r++) {
        if (wcell[r].second == 0)
            appendf(tail, "gstore(const_cast<uint64_t *>(p.cp[%u]) + i`, gl_canon(w%u`));\n", wcell[r].first, r);
        else
            appendf(tail, "gstore(const_cast<uint64_t *>(p.cp[%u]) + ((i` + (uint64_t)(%d)) & m), gl_canon(w%u`));\n",
                    wcell[r].first, wcell[r].second, r);
    }
    src += expand_rows(decl, rows);
    src += expand_rows(dot_decls, rows);
    src += expand_rows(body, rows);
    src += "}\n";
    if (kchunk) src += "if (live_) {\n";
    src += expand_rows(tail, rows);
    if (kchunk) src += "}\n";
    src += "#undef C\n}\n";
    return 0;
}

namespace {

// one kernel ready to launch: source, tables, compiled function
struct JitKernel {
    std::string src;
    std::vector<const uint64_t *> cp;
    std::vector<uint64_t> kc;
    std::vector<uint32_t> kl;
    std::vector<JitTerm> zt;
    hipFunction_t fn = nullptr;
    size_t off = 0, off_cp = 0, off_kc = 0, off_kl = 0, end = 0;  // table layout in the launch buffer
    bool klds = false;
    uint32_t rows = 1;  // rows per thread (ZKJIT_ROWS)
    double bytes = 0;
};

int prepare(const ZxpJitIn &in, JitKernel &K)
{
    K.cp.clear();
    K.kc.clear();
    K.kl.clear();
    K.zt.clear();
    const int rc = zxp_jit_build_source(in, K.src, K.cp, K.kc, K.kl, K.zt);
    const size_t at = K.src.find("#define ZKJIT_ROWS ");
    K.rows = at == std::string::npos ? 1 : (uint32_t)atoi(K.src.c_str() + at + 19);
    return rc;
}

// code objects of several sources (disk cache or hiprtc), compiled in
// parallel threads: the segments of a large program are independent
void objects_parallel(const std::vector<const std::string *> &srcs, std::vector<std::vector<char>> &code,
                      std::vector<int> &rcs, std::vector<uint8_t> *from_cache = nullptr)
{
    code.assign(srcs.size(), {});
    rcs.assign(srcs.size(), 0);
    if (from_cache) from_cache->assign(srcs.size(), 0);
    static const unsigned nthr = [] {
        const char *e = getenv("ZKGPU_ZXP_JIT_THREADS");
        const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
        return e && atoi(e) > 0 ? (unsigned)atoi(e) : std::min(16u, hc);
    }();
    std::vector<std::thread> th;
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (size_t j; (j = next++) < srcs.size();) {
            bool hit = false;
            rcs[j] = code_object(*srcs[j], code[j], &hit);
            if (from_cache) (*from_cache)[j] = hit;
        }
    };
    const unsigned n = std::min<unsigned>(nthr, (unsigned)srcs.size());
    for (unsigned t = 1; t < n; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
}

// code objects of several kernels: the ones not in this process's cache are
// found on disk or compiled by hiprtc, in parallel (the segments of a large
// program compile independently), then loaded
int compile_all(std::vector<JitKernel *> ks)
{
    Cache &c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    std::vector<JitKernel *> todo;
    for (JitKernel *k : ks) {
        auto it = c.fn.find(k->src);
        if (it != c.fn.end())
            k->fn = it->second;
        else if (std::find_if(todo.begin(), todo.end(), [&](JitKernel *t) { return t->src == k->src; }) == todo.end())
            todo.push_back(k);
    }
    std::vector<const std::string *> srcs;
    for (JitKernel *k : todo) srcs.push_back(&k->src);
    std::vector<std::vector<char>> code;
    std::vector<int> rcs;
    std::vector<uint8_t> hit;
    objects_parallel(srcs, code, rcs, &hit);
    for (size_t j = 0; j < todo.size(); j++) {
        int rc;
        if (rcs[j]) return rcs[j];
        hipModule_t mod;
        if (hit[j] && hipModuleLoadData(&mod, code[j].data()) != hipSuccess) {
            // a cached object the runtime refuses: a miss -- compile and replace it
            (void)hipGetLastError();
            if ((rc = rtc_compile(todo[j]->src, code[j]))) return rc;
            cache_store(todo[j]->src, code[j]);
            hit[j] = 0;
        }
        if (!hit[j] && (rc = check_hip(hipModuleLoadData(&mod, code[j].data()), "zxp jit: hipModuleLoadData")))
            return rc;
        hipFunction_t f;
        if ((rc = check_hip(hipModuleGetFunction(&f, mod, "zxp_jit"), "zxp jit: hipModuleGetFunction"))) return rc;
        c.fn.emplace(todo[j]->src, f);
    }
    for (JitKernel *k : ks) k->fn = c.fn.at(k->src);
    return 0;
}

// tables of every kernel in one buffer (zt | cp | kc | kl per kernel), one
// upload, then the launches in order on stream s
int launch_all(std::vector<JitKernel> &ks, const ZxpJitIn &in, hipStream_t s)
{
    size_t total = 0;
    for (JitKernel &K : ks) {
        K.off = total;
        K.off_cp = K.off + K.zt.size() * sizeof(JitTerm);
        K.off_kc = K.off_cp + K.cp.size() * 8;
        K.off_kl = (K.off_kc + (K.kc.size() + 1) * 8 + 15) & ~(size_t)15;  // 16-byte limb slots
        K.end = K.off_kl + (K.kl.size() + 1) * 4;
        total = (K.end + 15) & ~(size_t)15;
        K.klds = jit_kl_lds(K.kl.size()) && K.src.find("#define ZKJIT_KL_CHUNK 0") != std::string::npos;
    }
    // The tables go through a pinned staging buffer, so the upload is
    // asynchronous and the host does not wait for the stream's earlier work
    // (a stage's kernels queued before this program): the staging buffer is
    // rewritten only after its last upload has landed (event), and the
    // device buffer after the last kernels that read it (stream order, or an
    // event if the stream changed).
    static hipEvent_t up = nullptr, use = nullptr;
    static char *pin = nullptr;
    static size_t pin_cap = 0;
    int rc;
    if (!up && ((rc = check_hip(hipEventCreateWithFlags(&up, hipEventDisableTiming), "zxp jit: event")) ||
                (rc = check_hip(hipEventCreateWithFlags(&use, hipEventDisableTiming), "zxp jit: event"))))
        return rc;
    if ((rc = check_hip(hipEventSynchronize(up), "zxp jit: staging"))) return rc;
    if (total > pin_cap) {
        if (pin) (void)hipHostFree(pin);
        pin = nullptr;
        pin_cap = 0;
        if ((rc = check_hip(hipHostMalloc((void **)&pin, total), "zxp jit: staging buffer"))) return rc;
        pin_cap = total;
    }
    char *buf = jit_buf(total, use);
    if (!buf) return set_error(ZKGPU_ERR_OOM, "zxp jit: table buffer");
    memset(pin, 0, total);
    for (JitKernel &K : ks) {
        memcpy(pin + K.off, K.zt.data(), K.zt.size() * sizeof(JitTerm));
        memcpy(pin + K.off_cp, K.cp.data(), K.cp.size() * 8);
        memcpy(pin + K.off_kc, K.kc.data(), K.kc.size() * 8);
        memcpy(pin + K.off_kl, K.kl.data(), K.kl.size() * 4);
    }
    if ((rc = check_hip(hipStreamWaitEvent(s, use, 0), "zxp jit: table order"))) return rc;
    if ((rc = check_hip(hipMemcpyAsync(buf, pin, total, hipMemcpyHostToDevice, s), "zxp jit: H2D"))) return rc;
    if ((rc = check_hip(hipEventRecord(up, s), "zxp jit: event"))) return rc;
    Ctx &c = ctx();
    const uint64_t dom = 1ULL << in.log_dom;
    for (JitKernel &K : ks)
        if (dom < K.rows) return set_error(ZKGPU_ERR_ARG, "zxp jit: 2^%u rows < %u rows per thread", in.log_dom, K.rows);
    for (size_t j = 0; j < ks.size(); j++) {
        JitKernel &K = ks[j];
        JitParams p;
        p.zt = (const JitTerm *)(buf + K.off);
        p.cp = (const uint64_t *const *)(buf + K.off_cp);
        p.kc = (const uint64_t *)(buf + K.off_kc);
        p.kl = (const uint32_t *)(buf + K.off_kl);
        p.xdiv = in.xdiv;
        p.xdivw = in.xdivw;
        p.zh = in.zh_dev;
        p.tw_lo = c.tw_lo[0];
        p.tw_hi = c.tw_hi[0];
        p.x_start = in.x_start;
        p.logdom = in.log_dom;
        p.logomega = in.log_omega;
        p.rmask = in.wrap ? dom - 1 : ~0ULL;
        p.zmask = in.zmask;
        p.nkl = K.klds ? (uint32_t)K.kl.size() : 0;
        p.one = 1;
        void *args[] = {&p};
        prof_begin(s);
        rc = check_hip(hipModuleLaunchKernel(K.fn, (uint32_t)((dom / K.rows + JIT_THREADS - 1) / JIT_THREADS), 1, 1,
                                             JIT_THREADS, 1, 1, K.klds ? (uint32_t)(K.kl.size() * 4) : 0, s, args,
                                             nullptr),
                       "zxp jit: launch");
        char name[32];
        if (ks.size() > 1)
            snprintf(name, sizeof(name), "k_zxp_jit_s%02zu", j);  // one segment of a large program
        else
            snprintf(name, sizeof(name), "k_zxp_jit");
        prof_end(name, K.bytes, s);
        if (rc) return rc;
    }
    return check_hip(hipEventRecord(use, s), "zxp jit: event");
}

// Segments of a large program (csrc/zxp_segment.hpp): one per seg_cost of
// estimated VALU work for programs of >= seg_min compiled instructions.
uint32_t segments_for(const zxp_compiled &cp)
{
    constexpr uint64_t seg_cost = 50000;
    constexpr uint32_t seg_min = 2000;
    if (cp.n_instr < seg_min) return 1;
    uint64_t cost = 0;
    for (uint32_t k = 0; k < cp.n_instr; k++) cost += zxp_instr_cost(cp, k);
    return (uint32_t)std::max<uint64_t>(1, (cost + seg_cost / 2) / seg_cost);
}

// the kernels of a program: one, or one per segment (scratch(n) returns the
// carry columns' base for n columns of ld 2^log_dom)
// An unsigned field of a code object's AMDGPU metadata note (msgpack map:
// the key string, then its value), e.g. .private_segment_fixed_size (scratch
// bytes per lane: > 0 means the kernel spills), .vgpr_count, .agpr_count.
static uint64_t co_note(const std::vector<char> &code, const char *key)
{
    const size_t kn = strlen(key);
    for (size_t at = 0; at + kn + 1 < code.size(); at++) {
        if (memcmp(code.data() + at, key, kn)) continue;
        const uint8_t *v = (const uint8_t *)code.data() + at + kn;
        const size_t left = code.size() - at - kn;
        if (v[0] < 0x80) return v[0];                                   // positive fixint
        if (v[0] == 0xcc && left > 1) return v[1];                      // uint8
        if (v[0] == 0xcd && left > 2) return ((uint64_t)v[1] << 8) | v[2];  // uint16 (big endian)
        if (v[0] == 0xce && left > 4)
            return ((uint64_t)v[1] << 24) | ((uint64_t)v[2] << 16) | ((uint64_t)v[3] << 8) | v[4];
        return 0;
    }
    return 0;
}
static uint64_t co_scratch_bytes(const std::vector<char> &code) { return co_note(code, ".private_segment_fixed_size"); }

// occupancy decisions already taken in this process: first source -> waves
// (0: keep it), so repeated evaluations do not reread code objects
static std::mutex g_waves_mu;
static std::unordered_map<std::string, uint32_t> g_waves;
static bool waves_known(const std::string &src, uint32_t &w)
{
    std::lock_guard<std::mutex> lk(g_waves_mu);
    auto it = g_waves.find(src);
    if (it == g_waves.end()) return false;
    w = it->second;
    return true;
}
static void waves_remember(const std::string &src, uint32_t w)
{
    std::lock_guard<std::mutex> lk(g_waves_mu);
    g_waves[src] = w;
}

// The same decision of a whole (unsegmented) program keyed by its structure
// -- instructions, operands, the DOT terms' sources, the launch shape; never
// the coefficient or constant values -- so that a program evaluated every
// proof is generated once per evaluation instead of twice (first source, then
// the source at the chosen occupancy; config-4 quotient).  A key shared by two
// programs can only cost one of them its occupancy target, never a result.
static uint64_t structure_key(const ZxpJitIn &in)
{
    uint64_t h = 0x9E3779B97F4A7C15ULL;
    auto mix = [&](uint64_t w) {
        h = (h ^ w) * 0xBF58476D1CE4E5B9ULL;
        h ^= h >> 31;
    };
    for (uint32_t k = 0; k < in.n_instr; k++) {
        const zxp_instr &I = in.ins[k];
        mix((uint64_t)I.op << 32 | I.dst);
        mix((uint64_t)I.a << 32 | I.b);
        if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3)
            for (uint32_t t = I.a; t < I.a + I.b; t++) mix((uint64_t)in.terms[t].src << 32 | in.terms[t].comp);
    }
    for (uint32_t k = 0; k < in.n_opnd; k++) {
        const zxp_operand &o = in.opnd[k];
        mix((uint64_t)o.kind << 32 | o.a);
        mix((uint64_t)o.b << 32 | o.c);
    }
    mix((uint64_t)in.n_instr << 32 | in.n_opnd);
    mix((uint64_t)in.n_tmp1 << 32 | in.n_tmp3);
    mix((uint64_t)in.log_dom << 40 | (uint64_t)in.log_omega << 20 | in.wrap);
    mix((uint64_t)in.dot_loop_min << 32 | in.force_split);
    return h;
}
static std::unordered_map<uint64_t, uint32_t> g_waves_fp;

// may_compile = false (source / cache queries): the occupancy decisions use
// only code objects already on disk, and stop where one is missing
int build_kernels(const ZxpJitIn &in, std::vector<JitKernel> &ks, const std::function<uint64_t *(uint32_t)> &scratch,
                  int only = -1, bool may_compile = true)
{
    // code object of a source: 0 found / compiled, 1 not on disk (query mode), < 0 error
    auto object = [&](const std::string &src, std::vector<char> &code) -> int {
        if (may_compile) return code_object(src, code);
        return cache_load(src, code) ? 0 : 1;
    };
    zxp_compiled view;
    memset(&view, 0, sizeof(view));
    view.instr = in.ins;
    view.n_instr = in.n_instr;
    view.opnd = in.opnd;
    view.n_opnd = in.n_opnd;
    view.term = in.terms;
    view.n_tmp1 = in.n_tmp1;
    view.n_tmp3 = in.n_tmp3;
    const uint32_t nseg = in.n_opnd ? segments_for(view) : 1;
    int rc;
    ks.clear();
    if (nseg <= 1) {
        ks.resize(1);
        ks[0].bytes = in.bytes;
        const bool decide = in.waves_per_eu == 0 && only <= 0;
        const uint64_t fp = decide ? structure_key(in) : 0;
        if (decide) {
            uint32_t w = 0;
            bool hit;
            {
                std::lock_guard<std::mutex> lk(g_waves_mu);
                auto it = g_waves_fp.find(fp);
                hit = it != g_waves_fp.end();
                if (hit) w = it->second;
            }
            if (hit) {
                ZxpJitIn in2 = in;
                in2.waves_per_eu = w;
                return prepare(in2, ks[0]);
            }
        }
        if ((rc = prepare(in, ks[0]))) return rc;
        // A kernel the compiler leaves at 169-256 registers runs 2 waves per
        // SIMD and is latency-bound: compiled again with an occupancy target
        // of 3 (<= 168; config-4 quotient 186 VGPRs, 15.3 -> 12.7 ms); one
        // above 256 (1 wave, AGPRs: the reference's step2prev, 512 + spills)
        // with a target of 2.  Kernels at 3+ waves are left alone (a target
        // lets the scheduler spend registers: FRI polynomial 8.9 -> 9.2 ms),
        // as are block-split programs (registers bounded by their blocks).
        // Decided from the code object's metadata, so the prebuilt cache and
        // the run agree.
        if (decide) {
            uint32_t w = 0;
            if (ks[0].src.find("#define ZKJIT_SPLIT 1") == std::string::npos && !waves_known(ks[0].src, w)) {
                std::vector<char> code;
                if ((rc = object(ks[0].src, code))) return rc < 0 ? rc : 0;  // (query mode: undecided)
                const uint64_t regs = co_note(code, ".vgpr_count") + co_note(code, ".agpr_count");
                w = regs > 256 ? 2 : regs > 168 ? 3 : 0;
                waves_remember(ks[0].src, w);
            }
            {
                std::lock_guard<std::mutex> lk(g_waves_mu);
                g_waves_fp[fp] = w;
            }
            if (w) {
                ZxpJitIn in2 = in;
                in2.waves_per_eu = w;
                if ((rc = prepare(in2, ks[0]))) return rc;
            }
        }
        return 0;
    }
    std::vector<ZxpSegment> seg;
    uint32_t n_scratch = 0;
    if ((rc = zxp_segment(view, nseg, seg, n_scratch))) return rc;
    uint64_t *scr = scratch(std::max<uint32_t>(1, n_scratch));
    if (!scr) return ZKGPU_ERR_OOM;
    const uint64_t dom = 1ULL << in.log_dom;
    ks.resize(seg.size());
    // The segments are independent: their sources are generated (and their
    // occupancy decided) in parallel threads -- on the zkEVM-shaped quotient
    // ~10 ms of host work per segment, 8 segments, each proof (the GPU waits
    // for it).  The occupancy memo and the disk cache are thread-safe.
    auto one = [&](size_t j) -> int {
        int rc;
        ZxpJitIn J = in;
        J.ins = seg[j].instr.data();
        J.n_instr = (uint32_t)seg[j].instr.size();
        J.opnd = seg[j].opnd.data();
        J.n_opnd = (uint32_t)seg[j].opnd.size();
        J.terms = seg[j].term.data();
        J.force_split = 1;
        // occupancy target of a segment (seg_waves): 4 waves per SIMD (128
        // VGPRs; the 512-byte blocks keep fewer values live than the round-5
        // 1024-byte ones, which spilled up to 348 bytes with the prefetch).
        // A segment whose code spills more than spill_max bytes per lane
        // (300) at that target is compiled again one wave
        // lower (down to 2): the reference's step3 segments spill 324-452
        // bytes at 4 waves, none at 2.
        const uint32_t seg_waves = seg_ab().waves ? seg_ab().waves : 4;
        constexpr uint64_t spill_max = 300;
        const bool fixed = J.waves_per_eu != 0;
        J.scratch = scr;
        J.scratch_ld = dom;
        uint32_t w = fixed ? J.waves_per_eu : seg_waves;
        J.waves_per_eu = w;
        if ((rc = prepare(J, ks[j]))) return rc;  // 1: unsupported shape -> interpreter for the whole program
        if (!fixed && (only < 0 || (size_t)only == j)) {
            const std::string first = ks[j].src;
            uint32_t wk = 0;
            if (waves_known(first, wk)) {
                if (wk != w) {
                    J.waves_per_eu = wk;
                    if ((rc = prepare(J, ks[j]))) return rc;
                }
            } else {
                bool known = true;
                while (w > 2) {
                    std::vector<char> code;
                    if ((rc = object(ks[j].src, code)) < 0) return rc;
                    if (rc) {  // query mode, not compiled yet: undecided
                        known = false;
                        break;
                    }
                    if (co_scratch_bytes(code) <= spill_max) break;
                    J.waves_per_eu = --w;
                    if ((rc = prepare(J, ks[j]))) return rc;
                }
                if (known) waves_remember(first, w);
            }
        }
        ks[j].bytes = in.bytes / seg.size() + 8.0 * (seg[j].carry_in + seg[j].carry_out) * (double)dom;
        return 0;
    };
    std::vector<int> rcs(seg.size(), 0);
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (size_t j; (j = next++) < seg.size();) rcs[j] = one(j);
    };
    std::vector<std::thread> th;
    const size_t nthr = std::min<size_t>(seg.size(), std::max(1u, std::min(8u, std::thread::hardware_concurrency())));
    for (size_t t = 1; t < nthr; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    for (int r : rcs)
        if (r) return r;  // the first failing segment in order (1: unsupported shape -> the interpreter)
    return 0;
}

}  // namespace

int zxp_jit_run(const ZxpJitIn &in, hipStream_t s)
{
    std::vector<JitKernel> ks;
    int rc = build_kernels(in, ks, [&](uint32_t n) { return workspace(6, (size_t)n << in.log_dom << 3); });
    if (rc) return rc;
    std::vector<JitKernel *> pk;
    for (JitKernel &K : ks) pk.push_back(&K);
    if ((rc = compile_all(pk))) return rc;
    return launch_all(ks, in, s);
}

}  // namespace zk

// Diagnostics (C-ABI, include/zkgpu.h): compile a program as
// zkgpu_zxp_eval_dev would and print its straight-line kernel source;
// optionally run hiprtc on it.  No GPU needed.
extern "C" int zkgpu_zxp_jit_source(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd,
                                    uint32_t n_tmp1, uint32_t n_tmp3, const uint64_t *challenges,
                                    const uint64_t *publics, uint32_t n_publics, const uint64_t *evals,
                                    uint32_t n_evals, char *buf, uint64_t buflen, int rtc_check)
{
    using namespace zk;
    zxp_compiled cp;
    int rc = zkgpu_zxp_compile(instr, n_instr, opnd, n_opnd, n_tmp1, n_tmp3, challenges, publics, n_publics, evals,
                               n_evals, 0, &cp);
    if (rc) return rc;
    // placeholder sections: pointers are kernel inputs, not part of the source
    static uint64_t dummy;
    zkgpu_sections S;
    for (int k = 0; k < 12; k++) {
        S.sec[k] = &dummy;
        S.ld[k] = 1;
        S.ncols[k] = 0;
    }
    ZxpJitIn J;
    memset(&J, 0, sizeof(J));
    J.ins = cp.instr;
    J.n_instr = cp.n_instr;
    J.opnd = cp.opnd;
    J.terms = cp.term;
    J.csts = cp.cst;
    J.n_tmp1 = cp.n_tmp1;
    J.n_tmp3 = cp.n_tmp3;
    J.sections = &S;
    J.challenges = challenges;
    J.publics = publics;
    J.evals = evals;
    J.n_opnd = cp.n_opnd;
    // the same settings as zkgpu_zxp_eval_dev (api.hip), so the sources (and
    // cache keys) match
    J.dot_loop_min = 8;
    J.waves_per_eu = 0;
    std::vector<JitKernel> ks;
    static uint64_t dummy_scratch;
    const char *only_env = getenv("ZKGPU_ZXP_JIT_ONLY");
    if ((rc = build_kernels(J, ks, [](uint32_t) { return &dummy_scratch; }, only_env ? atoi(only_env) : -1,
                            rtc_check == 1 || rtc_check == 2)))
        return rc < 0 ? rc : set_error(ZKGPU_ERR_ARG, "zxp jit: unsupported program shape");
    std::string src;  // the kernels' sources (one per segment)
    for (size_t j = 0; j < ks.size(); j++) {
        if (ks.size() > 1) appendf(src, "// ---- segment %zu of %zu\n", j, ks.size());
        src += ks[j].src;
    }
    if (buf && buflen) {
        const size_t n = std::min<size_t>(src.size(), buflen - 1);
        memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    if (rtc_check == 3) {  // cache query only: 1 = every compiled object on disk
        std::vector<char> code;
        for (const JitKernel &K : ks)
            if (!cache_load(K.src, code)) return 0;
        return 1;
    }
    if (rtc_check) {
        // compile (or find in the disk cache); rtc_check == 2 also writes the
        // code objects to $ZKGPU_ZXP_JIT_DUMP (.<segment> appended when there
        // are several; register / scratch inspection)
        // ZKGPU_ZXP_JIT_ONLY=j: only segment j (tools/jit_prebuild.py runs the
        // segments in parallel processes: hiprtc serialises threads)
        std::vector<const std::string *> srcs;
        std::vector<size_t> idx;
        const char *only = getenv("ZKGPU_ZXP_JIT_ONLY");
        for (size_t j = 0; j < ks.size(); j++)
            if (!only || (size_t)atoi(only) == j) {
                srcs.push_back(&ks[j].src);
                idx.push_back(j);
            }
        std::vector<std::vector<char>> code;
        std::vector<int> rcs;
        objects_parallel(srcs, code, rcs);
        for (int r : rcs)
            if (r) return r;
        const char *dump = getenv("ZKGPU_ZXP_JIT_DUMP");
        if (rtc_check == 2 && dump)
            for (size_t j = 0; j < code.size(); j++) {
                const std::string path = ks.size() > 1 ? std::string(dump) + "." + std::to_string(idx[j]) : dump;
                FILE *f = fopen(path.c_str(), "wb");
                if (f) {
                    fwrite(code[j].data(), 1, code[j].size(), f);
                    fclose(f);
                }
            }
    }
    return (int)std::min<size_t>(src.size(), 0x7FFFFFFF);
}
