// Plookup h1/h2 columns on the GPU: Polinomial::calculateH1H2_opt1 (dim 1,
// polinomial.hpp:349-463) / calculateH1H2_opt3 (dim 3, :465-583), called per
// plookup from Starks::genProof stage 2 (starks.cpp:104-127).
//
// The reference builds a chained hash table of the table column t (each key
// remembers its LAST row), counts every f value onto that row, and deals the
// resulting multiset (t[j] repeated 1 + count_j times, in t order) alternately
// into h1 and h2.  The same mapping, data-parallel (h1h2_hash): an
// open-addressing table of table ROWS keyed by the canonical value (linear
// probing, 2^k >= 2N slots of u32): insertion keeps the largest row per key
// (atomicMax: the reference's "last row wins"), every f row probes and counts
// onto its row (counts start at 1; an absent key records the smallest such f
// row, "Number not included"), an exclusive scan of the counts gives each
// table row its start in the 2N-long multiset, and one thread per table row
// scatters its 1 + count raw copies (copyElement) alternately into h1 / h2.
// Columns are column-major: component c of a dim-3 column at ptr + c * ld.
// (A stable radix sort of the keys with a two-level upper_bound was the
// round-2 form: 8.1 against 1.9 ms for two plookups at 2^23.)
#include <stdlib.h>

#include <vector>

#include <rocprim/device/device_scan.hpp>

#include "gl_device.hpp"
#include "zkgpu_internal.hpp"

namespace zk {

static inline uint32_t nblk2(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

__global__ void k_h12_fill1(uint32_t *c, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) c[i] = 1;
}

// ---------------------------------------------------------------- hash path
constexpr uint32_t H12_EMPTY = 0xFFFFFFFFu;

template <int DIM>
__device__ __forceinline__ void h12_key(uint64_t key[DIM], const uint64_t *col, uint64_t ld, uint64_t r)
{
#pragma unroll
    for (int c = 0; c < DIM; c++) key[c] = gl_canon(col[c * ld + r]);
}

template <int DIM>
__device__ __forceinline__ uint64_t h12_hash(const uint64_t key[DIM])
{
    uint64_t h = 0x9E3779B97F4A7C15ULL;
#pragma unroll
    for (int c = 0; c < DIM; c++) {
        uint64_t z = key[c] + h;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        h = z ^ (z >> 31);
    }
    return h;
}

template <int DIM>
__device__ __forceinline__ bool h12_eq(const uint64_t *t, uint64_t t_ld, uint32_t row, const uint64_t key[DIM])
{
#pragma unroll
    for (int c = 0; c < DIM; c++)
        if (gl_canon(t[c * t_ld + row]) != key[c]) return false;
    return true;
}

// table row i -> its key's slot holds the largest row with that key
template <int DIM>
__global__ void __launch_bounds__(256) k_h12_insert(uint32_t *slots, uint64_t mask, const uint64_t *t, uint64_t t_ld,
                                                    uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t key[DIM];
    h12_key<DIM>(key, t, t_ld, i);
    uint64_t h = h12_hash<DIM>(key) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        uint32_t cur = slots[h];
        if (cur == H12_EMPTY) {
            cur = atomicCAS(&slots[h], H12_EMPTY, (uint32_t)i);
            if (cur == H12_EMPTY) return;
        }
        if (h12_eq<DIM>(t, t_ld, cur, key)) {
            atomicMax(&slots[h], (uint32_t)i);
            return;
        }
    }
}

// f row i -> ++cnt[last table row with f's key]; absent keys record the
// smallest such row
template <int DIM>
__global__ void __launch_bounds__(256) k_h12_probe(const uint32_t *slots, uint64_t mask, const uint64_t *f,
                                                   uint64_t f_ld, const uint64_t *t, uint64_t t_ld, uint64_t n,
                                                   uint32_t *cnt, unsigned long long *miss)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t key[DIM];
    h12_key<DIM>(key, f, f_ld, i);
    uint64_t h = h12_hash<DIM>(key) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        const uint32_t cur = slots[h];
        if (cur == H12_EMPTY) break;
        if (h12_eq<DIM>(t, t_ld, cur, key)) {
            atomicAdd(&cnt[cur], 1u);
            return;
        }
    }
    atomicMin(miss, (unsigned long long)i);
}

// table row j: its 1 + count copies at multiset slots start[j] ..
template <int DIM>
__global__ void __launch_bounds__(256) k_h12_scatter(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld,
                                                     const uint64_t *t, uint64_t t_ld, const uint32_t *start,
                                                     const uint32_t *cnt, uint64_t n)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint64_t v[DIM];
#pragma unroll
    for (int c = 0; c < DIM; c++) v[c] = t[c * t_ld + j];  // raw copy (copyElement)
    const uint64_t s0 = start[j], e = s0 + cnt[j];
    for (uint64_t sl = s0; sl < e; sl++) {
        uint64_t *h = (sl & 1) ? h2 : h1;
        const uint64_t ld = (sl & 1) ? h2_ld : h1_ld;
#pragma unroll
        for (int c = 0; c < DIM; c++) h[c * ld + (sl >> 1)] = v[c];
    }
}

static int h1h2_hash(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *f, uint64_t f_ld,
                     const uint64_t *t, uint64_t t_ld, uint64_t n, uint32_t dim, uint64_t *missing_row, hipStream_t s)
{
    uint64_t m = 1;
    while (m < 2 * n) m <<= 1;
    const size_t need = m * 4 + 2 * n * 4 + 16;
    char *w = (char *)workspace(4, need);
    if (!w) return ZKGPU_ERR_OOM;
    uint32_t *slots = (uint32_t *)w;
    uint32_t *cnt = slots + m;
    uint32_t *start = cnt + n;
    unsigned long long *miss = (unsigned long long *)(((uintptr_t)(start + n) + 7) & ~(uintptr_t)7);
    size_t scan_bytes = 0;
    if (rocprim::exclusive_scan(nullptr, scan_bytes, cnt, start, 0u, (size_t)n, rocprim::plus<uint32_t>(), s) !=
        hipSuccess)
        return set_error(ZKGPU_ERR_HIP, "h1h2: rocprim temp-size query failed");
    void *tmp = workspace(5, scan_bytes);
    if (!tmp) return ZKGPU_ERR_OOM;
    const uint32_t B = 256;
    prof_begin(s);
    if (check_hip(hipMemsetAsync(slots, 0xFF, m * 4, s), "h1h2 memset") ||
        check_hip(hipMemsetAsync(miss, 0xFF, 8, s), "h1h2 memset"))
        return ZKGPU_ERR_HIP;
    hipLaunchKernelGGL(k_h12_fill1, dim3(nblk2(n, B)), dim3(B), 0, s, cnt, n);
    if (dim == 1) {
        hipLaunchKernelGGL(k_h12_insert<1>, dim3(nblk2(n, B)), dim3(B), 0, s, slots, m - 1, t, t_ld, n);
        hipLaunchKernelGGL(k_h12_probe<1>, dim3(nblk2(n, B)), dim3(B), 0, s, slots, m - 1, f, f_ld, t, t_ld, n, cnt,
                           miss);
    } else {
        hipLaunchKernelGGL(k_h12_insert<3>, dim3(nblk2(n, B)), dim3(B), 0, s, slots, m - 1, t, t_ld, n);
        hipLaunchKernelGGL(k_h12_probe<3>, dim3(nblk2(n, B)), dim3(B), 0, s, slots, m - 1, f, f_ld, t, t_ld, n, cnt,
                           miss);
    }
    {
        size_t tb = scan_bytes;
        if (rocprim::exclusive_scan(tmp, tb, cnt, start, 0u, (size_t)n, rocprim::plus<uint32_t>(), s) != hipSuccess)
            return set_error(ZKGPU_ERR_HIP, "h1h2: scan failed");
    }
    unsigned long long mh = 0;
    if (check_hip(hipMemcpyAsync(&mh, miss, 8, hipMemcpyDeviceToHost, s), "D2H") ||
        check_hip(hipStreamSynchronize(s), "h1h2 sync"))
        return ZKGPU_ERR_HIP;
    if (mh != ~0ULL) {
        if (missing_row) *missing_row = mh;
        return set_error(ZKGPU_ERR_ARG, "calculateH1H2: Number not included: w=%llu", mh);
    }
    if (missing_row) *missing_row = ~0ULL;
    if (dim == 1)
        hipLaunchKernelGGL(k_h12_scatter<1>, dim3(nblk2(n, B)), dim3(B), 0, s, h1, h1_ld, h2, h2_ld, t, t_ld, start, cnt,
                           n);
    else
        hipLaunchKernelGGL(k_h12_scatter<3>, dim3(nblk2(n, B)), dim3(B), 0, s, h1, h1_ld, h2, h2_ld, t, t_ld, start, cnt,
                           n);
    prof_end("k_h1h2", (double)dim * 8.0 * 4.0 * n, s);
    return check_launch("h1h2");
}

int h1h2(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *f, uint64_t f_ld,
         const uint64_t *t, uint64_t t_ld, uint64_t n, uint32_t dim, uint64_t *missing_row, hipStream_t s)
{
    return h1h2_hash(h1, h1_ld, h2, h2_ld, f, f_ld, t, t_ld, n, dim, missing_row, s);
}

// ---------------------------------------------------------------- row-sharded
// calculateH1H2 over W ranks, each holding rows [row0, row0 + n) of f and t
// (host/sharded_starks.hpp h1h2_all).  The mapping is the one above: table
// row j appears 1 + count_j times in the multiset (count_j = the f rows with
// t[j]'s key, on the LAST table row with that key, else 0), in table order,
// dealt alternately into h1 / h2.  Split as:
//   route   each rank dedupes its rows: distinct t keys with their largest
//           row, distinct f keys with their count and smallest row; each
//           distinct key goes to the rank owning hash(key) as a record
//           {k0, k1, k2, global row, val} (val = H12S_T for a t key, the f
//           count otherwise), bucketed by owner, t records first
//   owner   per key: the largest t row over all ranks, the f counts summed;
//           f keys with no t row give the smallest such f row (the
//           reference's "Number not included"); returns, aligned with the t
//           records, the count for the winning row (0 for the others)
//   counts  the sender: count_j = 1 + returned count of row j; exclusive
//           scan -> the rank's multiset positions, relative to its offset
//   deal    the rank's segment of the multiset (its table rows' copies)
//   place   a received piece of the multiset into the rank's h1 / h2 rows
constexpr uint64_t H12S_T = ~0ULL;
constexpr int H12S_REC = 5;  // words per record

__device__ __forceinline__ uint32_t h12s_owner(uint64_t h, uint32_t world)
{
    return (uint32_t)(((h >> 32) * (uint64_t)world) >> 32);  // high hash bits (the table probes use the low ones)
}

// local f table: slot -> smallest row with the key, fcnt[slot] = its rows
template <int DIM>
__global__ void __launch_bounds__(256) k_h12s_insert_f(uint32_t *slots, uint32_t *fcnt, uint64_t mask,
                                                       const uint64_t *f, uint64_t f_ld, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t key[DIM];
    h12_key<DIM>(key, f, f_ld, i);
    uint64_t h = h12_hash<DIM>(key) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        uint32_t cur = slots[h];
        if (cur == H12_EMPTY) {
            cur = atomicCAS(&slots[h], H12_EMPTY, (uint32_t)i);
            if (cur == H12_EMPTY) {
                atomicAdd(&fcnt[h], 1u);
                return;
            }
        }
        if (h12_eq<DIM>(f, f_ld, cur, key)) {  // every row a slot ever holds has its key
            atomicMin(&slots[h], (uint32_t)i);
            atomicAdd(&fcnt[h], 1u);
            return;
        }
    }
}

// records of the occupied slots of the local t table (tab 0) and f table
// (tab 1): count per owner (pass 0) or write into the owner's bucket (pass 1)
template <int DIM>
__global__ void __launch_bounds__(256) k_h12s_bucket(uint64_t *recs, const uint32_t *tslots, const uint32_t *fslots,
                                                     const uint32_t *fcnt, uint64_t m, const uint64_t *t, uint64_t t_ld,
                                                     const uint64_t *f, uint64_t f_ld, uint64_t row0, uint32_t world,
                                                     uint32_t *cnt /* 2 W */, const uint64_t *base /* 2 W */,
                                                     int pass)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= 2 * m) return;
    const int tab = k >= m;
    const uint64_t sl = tab ? k - m : k;
    const uint32_t row = tab ? fslots[sl] : tslots[sl];
    if (row == H12_EMPTY) return;
    uint64_t key[DIM];
    h12_key<DIM>(key, tab ? f : t, tab ? f_ld : t_ld, row);
    const uint32_t o = h12s_owner(h12_hash<DIM>(key), world);
    const uint32_t pos = atomicAdd(&cnt[2 * o + tab], 1u);
    if (!pass) return;
    uint64_t *r = recs + (base[2 * o + tab] + pos) * H12S_REC;
#pragma unroll
    for (int c = 0; c < 3; c++) r[c] = c < DIM ? key[c] : 0;
    r[3] = row0 + row;
    r[4] = tab ? (uint64_t)fcnt[sl] : H12S_T;
}

template <int DIM>
__device__ __forceinline__ void h12s_rkey(uint64_t key[DIM], const uint64_t *r)
{
#pragma unroll
    for (int c = 0; c < DIM; c++) key[c] = r[c];
}

template <int DIM>
__device__ __forceinline__ bool h12s_req(const uint64_t *r, const uint64_t key[DIM])
{
#pragma unroll
    for (int c = 0; c < DIM; c++)
        if (r[c] != key[c]) return false;
    return true;
}

// owner: t records -> slot = ((row + 1) << 32 | record), largest row wins
template <int DIM>
__global__ void __launch_bounds__(256) k_h12s_own_insert(unsigned long long *slots, uint64_t mask, const uint64_t *recs,
                                                         uint64_t nrec)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nrec) return;
    const uint64_t *r = recs + k * H12S_REC;
    if (r[4] != H12S_T) return;
    uint64_t key[DIM];
    h12s_rkey<DIM>(key, r);
    const unsigned long long mine = ((unsigned long long)(r[3] + 1) << 32) | k;
    uint64_t h = h12_hash<DIM>(key) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        unsigned long long cur = slots[h];
        if (!cur) {
            cur = atomicCAS(&slots[h], 0ULL, mine);
            if (!cur) return;
        }
        if (h12s_req<DIM>(recs + (cur & 0xFFFFFFFFULL) * H12S_REC, key)) {
            atomicMax(&slots[h], mine);
            return;
        }
    }
}

template <int DIM>
__device__ __forceinline__ uint64_t h12s_find(const unsigned long long *slots, uint64_t mask, const uint64_t *recs,
                                              const uint64_t key[DIM])
{
    uint64_t h = h12_hash<DIM>(key) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        const unsigned long long cur = slots[h];
        if (!cur) break;
        if (h12s_req<DIM>(recs + (cur & 0xFFFFFFFFULL) * H12S_REC, key)) return cur & 0xFFFFFFFFULL;
    }
    return ~0ULL;
}

// owner: f records -> the winning t record's sum; absent keys: smallest row
template <int DIM>
__global__ void __launch_bounds__(256) k_h12s_own_probe(const unsigned long long *slots, uint64_t mask,
                                                        const uint64_t *recs, uint64_t nrec,
                                                        unsigned long long *sum, unsigned long long *miss)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nrec) return;
    const uint64_t *r = recs + k * H12S_REC;
    if (r[4] == H12S_T) return;
    uint64_t key[DIM];
    h12s_rkey<DIM>(key, r);
    const uint64_t w = h12s_find<DIM>(slots, mask, recs, key);
    if (w == ~0ULL)
        atomicMin(miss, (unsigned long long)r[3]);
    else
        atomicAdd(&sum[w], (unsigned long long)r[4]);
}

// owner: the return value of each t record (its count if it won its key)
template <int DIM>
__global__ void __launch_bounds__(256) k_h12s_own_ret(uint64_t *ret, const unsigned long long *slots, uint64_t mask,
                                                      const uint64_t *recs, uint64_t nrec,
                                                      const unsigned long long *sum)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nrec) return;
    const uint64_t *r = recs + k * H12S_REC;
    if (r[4] != H12S_T) {
        ret[k] = 0;
        return;
    }
    uint64_t key[DIM];
    h12s_rkey<DIM>(key, r);
    ret[k] = h12s_find<DIM>(slots, mask, recs, key) == k ? sum[k] : 0;
}

// sender: count_j = 1 + the count returned for row j's record
__global__ void k_h12s_apply(uint32_t *cnt, const uint64_t *sent, const uint64_t *ret, uint64_t nsent, uint64_t row0)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nsent) return;
    const uint64_t *r = sent + k * H12S_REC;
    if (r[4] == H12S_T && ret[k]) cnt[r[3] - row0] += (uint32_t)ret[k];  // one record per row: no race
}

// the rank's multiset segment: table row j's copies at start[j] .. (raw, like copyElement)
template <int DIM>
__global__ void __launch_bounds__(256) k_h12s_deal(uint64_t *seg, uint64_t seg_ld, const uint64_t *t, uint64_t t_ld,
                                                   const uint32_t *start, const uint32_t *cnt, uint64_t n)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint64_t v[DIM];
#pragma unroll
    for (int c = 0; c < DIM; c++) v[c] = t[c * t_ld + j];
    const uint64_t s0 = start[j], e = s0 + cnt[j];
    for (uint64_t p = s0; p < e; p++)
#pragma unroll
        for (int c = 0; c < DIM; c++) seg[c * seg_ld + p] = v[c];
}

// multiset positions [pos0, pos0 + len) (buf column-major, ld buf_ld) ->
// h1 (even positions) / h2 (odd) at local row p / 2 - row0
template <int DIM>
__global__ void __launch_bounds__(256) k_h12s_place(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld,
                                                    const uint64_t *buf, uint64_t buf_ld, uint64_t pos0, uint64_t len,
                                                    uint64_t row0)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= len) return;
    const uint64_t p = pos0 + k;
    uint64_t *h = (p & 1) ? h2 : h1;
    const uint64_t ld = (p & 1) ? h2_ld : h1_ld;
#pragma unroll
    for (int c = 0; c < DIM; c++) h[c * ld + (p >> 1) - row0] = buf[c * buf_ld + k];
}

static uint64_t h12s_table_size(uint64_t n)
{
    uint64_t m = 1;
    while (m < 2 * n) m <<= 1;
    return m;
}

int h1h2_shard_route(uint64_t *recs, uint64_t cap, uint32_t *n_t, uint32_t *n_f, const uint64_t *f, uint64_t f_ld,
                     const uint64_t *t, uint64_t t_ld, uint64_t n, uint64_t row0, uint32_t dim, uint32_t world,
                     hipStream_t s)
{
    const uint64_t m = h12s_table_size(n);
    const size_t need = 3 * m * 4 + 2ULL * world * 4 + 2ULL * world * 8 + 64;
    char *w = (char *)workspace(4, need);
    if (!w) return ZKGPU_ERR_OOM;
    uint32_t *tslots = (uint32_t *)w, *fslots = tslots + m, *fcnt = fslots + m, *cnt = fcnt + m;
    uint64_t *base = (uint64_t *)(((uintptr_t)(cnt + 2 * world) + 7) & ~(uintptr_t)7);
    const uint32_t B = 256;
    prof_begin(s);
    if (check_hip(hipMemsetAsync(tslots, 0xFF, 2 * m * 4, s), "h1h2 memset") ||
        check_hip(hipMemsetAsync(fcnt, 0, m * 4 + 2ULL * world * 4, s), "h1h2 memset"))
        return ZKGPU_ERR_HIP;
    if (dim == 1) {
        hipLaunchKernelGGL(k_h12_insert<1>, dim3(nblk2(n, B)), dim3(B), 0, s, tslots, m - 1, t, t_ld, n);
        hipLaunchKernelGGL(k_h12s_insert_f<1>, dim3(nblk2(n, B)), dim3(B), 0, s, fslots, fcnt, m - 1, f, f_ld, n);
        hipLaunchKernelGGL(k_h12s_bucket<1>, dim3(nblk2(2 * m, B)), dim3(B), 0, s, recs, tslots, fslots, fcnt, m, t,
                           t_ld, f, f_ld, row0, world, cnt, (const uint64_t *)base, 0);
    } else {
        hipLaunchKernelGGL(k_h12_insert<3>, dim3(nblk2(n, B)), dim3(B), 0, s, tslots, m - 1, t, t_ld, n);
        hipLaunchKernelGGL(k_h12s_insert_f<3>, dim3(nblk2(n, B)), dim3(B), 0, s, fslots, fcnt, m - 1, f, f_ld, n);
        hipLaunchKernelGGL(k_h12s_bucket<3>, dim3(nblk2(2 * m, B)), dim3(B), 0, s, recs, tslots, fslots, fcnt, m, t,
                           t_ld, f, f_ld, row0, world, cnt, (const uint64_t *)base, 0);
    }
    std::vector<uint32_t> c(2 * world);
    if (check_hip(hipMemcpyAsync(c.data(), cnt, 2ULL * world * 4, hipMemcpyDeviceToHost, s), "D2H") ||
        check_hip(hipStreamSynchronize(s), "h1h2 sync"))
        return ZKGPU_ERR_HIP;
    // buckets in owner order, t records first in each
    std::vector<uint64_t> b(2 * world);
    uint64_t off = 0;
    for (uint32_t o = 0; o < world; o++) {
        n_t[o] = c[2 * o];
        n_f[o] = c[2 * o + 1];
        b[2 * o] = off;
        b[2 * o + 1] = off + c[2 * o];
        off += (uint64_t)c[2 * o] + c[2 * o + 1];
    }
    if (off > cap)
        return set_error(ZKGPU_ERR_ARG, "h1h2 (sharded): %llu records exceed the %llu-record buffer",
                         (unsigned long long)off, (unsigned long long)cap);
    if (check_hip(hipMemcpyAsync(base, b.data(), 2ULL * world * 8, hipMemcpyHostToDevice, s), "H2D") ||
        check_hip(hipMemsetAsync(cnt, 0, 2ULL * world * 4, s), "h1h2 memset"))
        return ZKGPU_ERR_HIP;
    if (dim == 1)
        hipLaunchKernelGGL(k_h12s_bucket<1>, dim3(nblk2(2 * m, B)), dim3(B), 0, s, recs, tslots, fslots, fcnt, m, t,
                           t_ld, f, f_ld, row0, world, cnt, (const uint64_t *)base, 1);
    else
        hipLaunchKernelGGL(k_h12s_bucket<3>, dim3(nblk2(2 * m, B)), dim3(B), 0, s, recs, tslots, fslots, fcnt, m, t,
                           t_ld, f, f_ld, row0, world, cnt, (const uint64_t *)base, 1);
    if (check_hip(hipStreamSynchronize(s), "h1h2 sync")) return ZKGPU_ERR_HIP;  // b dies here
    prof_end("k_h1h2_route", (double)dim * 8.0 * 2.0 * n, s);
    return check_launch("h1h2 route");
}

int h1h2_shard_owner(uint64_t *ret, const uint64_t *recs, uint64_t nrec, uint32_t dim, uint64_t *miss_row,
                     hipStream_t s)
{
    const uint64_t m = h12s_table_size(nrec);
    const size_t need = m * 8 + nrec * 8 + 16;
    char *w = (char *)workspace(4, need);
    if (!w) return ZKGPU_ERR_OOM;
    unsigned long long *slots = (unsigned long long *)w, *sum = slots + m, *miss = sum + nrec;
    const uint32_t B = 256;
    prof_begin(s);
    if (check_hip(hipMemsetAsync(slots, 0, (m + nrec) * 8, s), "h1h2 memset") ||
        check_hip(hipMemsetAsync(miss, 0xFF, 8, s), "h1h2 memset"))
        return ZKGPU_ERR_HIP;
    if (nrec) {
        if (dim == 1) {
            hipLaunchKernelGGL(k_h12s_own_insert<1>, dim3(nblk2(nrec, B)), dim3(B), 0, s, slots, m - 1, recs, nrec);
            hipLaunchKernelGGL(k_h12s_own_probe<1>, dim3(nblk2(nrec, B)), dim3(B), 0, s, slots, m - 1, recs, nrec, sum,
                               miss);
            hipLaunchKernelGGL(k_h12s_own_ret<1>, dim3(nblk2(nrec, B)), dim3(B), 0, s, ret, slots, m - 1, recs, nrec,
                               sum);
        } else {
            hipLaunchKernelGGL(k_h12s_own_insert<3>, dim3(nblk2(nrec, B)), dim3(B), 0, s, slots, m - 1, recs, nrec);
            hipLaunchKernelGGL(k_h12s_own_probe<3>, dim3(nblk2(nrec, B)), dim3(B), 0, s, slots, m - 1, recs, nrec, sum,
                               miss);
            hipLaunchKernelGGL(k_h12s_own_ret<3>, dim3(nblk2(nrec, B)), dim3(B), 0, s, ret, slots, m - 1, recs, nrec,
                               sum);
        }
    }
    unsigned long long mh = 0;
    if (check_hip(hipMemcpyAsync(&mh, miss, 8, hipMemcpyDeviceToHost, s), "D2H") ||
        check_hip(hipStreamSynchronize(s), "h1h2 sync"))
        return ZKGPU_ERR_HIP;
    *miss_row = mh;
    prof_end("k_h1h2_owner", 40.0 * (double)nrec, s);
    return check_launch("h1h2 owner");
}

int h1h2_shard_counts(uint32_t *start, uint32_t *cnt, uint64_t *total, const uint64_t *sent, const uint64_t *ret,
                      uint64_t nsent, uint64_t n, uint64_t row0, hipStream_t s)
{
    size_t scan_bytes = 0;
    if (rocprim::exclusive_scan(nullptr, scan_bytes, cnt, start, 0u, (size_t)n, rocprim::plus<uint32_t>(), s) !=
        hipSuccess)
        return set_error(ZKGPU_ERR_HIP, "h1h2: rocprim temp-size query failed");
    void *tmp = workspace(5, scan_bytes);
    if (!tmp) return ZKGPU_ERR_OOM;
    const uint32_t B = 256;
    hipLaunchKernelGGL(k_h12_fill1, dim3(nblk2(n, B)), dim3(B), 0, s, cnt, n);
    if (nsent) hipLaunchKernelGGL(k_h12s_apply, dim3(nblk2(nsent, B)), dim3(B), 0, s, cnt, sent, ret, nsent, row0);
    size_t tb = scan_bytes;
    if (rocprim::exclusive_scan(tmp, tb, cnt, start, 0u, (size_t)n, rocprim::plus<uint32_t>(), s) != hipSuccess)
        return set_error(ZKGPU_ERR_HIP, "h1h2: scan failed");
    uint32_t last[2] = {0, 0};
    if (check_hip(hipMemcpyAsync(&last[0], start + n - 1, 4, hipMemcpyDeviceToHost, s), "D2H") ||
        check_hip(hipMemcpyAsync(&last[1], cnt + n - 1, 4, hipMemcpyDeviceToHost, s), "D2H") ||
        check_hip(hipStreamSynchronize(s), "h1h2 sync"))
        return ZKGPU_ERR_HIP;
    *total = (uint64_t)last[0] + last[1];
    return check_launch("h1h2 counts");
}

int h1h2_shard_deal(uint64_t *seg, uint64_t seg_ld, const uint64_t *t, uint64_t t_ld, const uint32_t *start,
                    const uint32_t *cnt, uint64_t n, uint32_t dim, hipStream_t s)
{
    const uint32_t B = 256;
    if (dim == 1)
        hipLaunchKernelGGL(k_h12s_deal<1>, dim3(nblk2(n, B)), dim3(B), 0, s, seg, seg_ld, t, t_ld, start, cnt, n);
    else
        hipLaunchKernelGGL(k_h12s_deal<3>, dim3(nblk2(n, B)), dim3(B), 0, s, seg, seg_ld, t, t_ld, start, cnt, n);
    return check_launch("h1h2 deal");
}

int h1h2_shard_place(uint64_t *h1, uint64_t h1_ld, uint64_t *h2, uint64_t h2_ld, const uint64_t *buf, uint64_t buf_ld,
                     uint64_t pos0, uint64_t len, uint64_t row0, uint32_t dim, hipStream_t s)
{
    if (!len) return 0;
    const uint32_t B = 256;
    if (dim == 1)
        hipLaunchKernelGGL(k_h12s_place<1>, dim3(nblk2(len, B)), dim3(B), 0, s, h1, h1_ld, h2, h2_ld, buf, buf_ld, pos0,
                           len, row0);
    else
        hipLaunchKernelGGL(k_h12s_place<3>, dim3(nblk2(len, B)), dim3(B), 0, s, h1, h1_ld, h2, h2_ld, buf, buf_ld, pos0,
                           len, row0);
    return check_launch("h1h2 place");
}

}  // namespace zk
