// libzkgpu_stark: the host-side STARK prover on top of the libzkgpu C-ABI.
//
// A C++ restatement of the reference's host orchestration -- Starks::genProof
// (src/starkpil/starks.cpp:9-404), FRIProve::prove / queryPol
// (src/starkpil/fri/friProve.cpp:5-232) and Transcript
// (src/starkpil/transcript/transcript.cpp:4-87) -- in which every bulk
// operation is a device-resident libzkgpu call on column-major sections kept
// in HBM for the whole proof.  Only roots, evals, challenges, query openings
// and the final polynomial cross PCIe.  Host arithmetic is limited to the
// scalars the reference also computes on the host (challenge transforms,
// shift powers, zhInv table size), done with the 128-bit helpers below.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <string>
#include <vector>

#include "../../include/zkgpu.h"
#include "../../include/zkgpu_stark.h"

namespace zkgpu_host {

static thread_local char g_err[512] = "";
static int fail(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return -1;
}
// the message of the last fail() on this thread (e.g. a communicator's, before
// the prover's own wraps it)
static std::string last_error_text() { return g_err; }
#define CK(x)                                                                                                  \
    do {                                                                                                       \
        int _rc = (x);                                                                                         \
        if (_rc) return fail("%s: %s (%s:%d)", #x, zkgpu_last_error(), __FILE__, __LINE__);                   \
    } while (0)

static const uint64_t P = 0xFFFFFFFF00000001ULL;
static uint64_t mul(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) % P); }
static uint64_t pw(uint64_t a, uint64_t e)
{
    uint64_t r = 1;
    a %= P;
    while (e) {
        if (e & 1) r = mul(r, a);
        a = mul(a, a);
        e >>= 1;
    }
    return r;
}
static uint64_t inv(uint64_t a) { return pw(a, P - 2); }
static uint64_t w_of(uint32_t n)  // Goldilocks::w(n)
{
    uint64_t w = 7277203076849721926ULL;
    for (uint32_t i = n; i < 32; i++) w = mul(w, w);
    return w;
}
static uint64_t rand_u64(uint64_t seed, uint64_t stream, uint64_t col, uint64_t row)
{
    uint64_t x = seed ^ (stream << 56) ^ (col * 0x9E3779B97F4A7C15ULL) ^ (row * 0xC2B2AE3D27D4EB4FULL);
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return z >> 1;
}

// ---------------------------------------------------------------- transcript
// The transcript runs on the host, as the reference's (transcript.cpp:4-87):
// its permutations are a serial chain on the critical path between stages, so
// they use the host permutation zkgpu_gl_poseidon_full_host (~5 us) rather
// than a single-thread GPU launch plus a synchronisation (~70 us, 90 per proof).
// Transcript (transcript.cpp:4-87)
class Transcript
{
public:
    uint64_t state[4] = {0, 0, 0, 0};
    uint64_t pending[8] = {0};
    uint64_t out[12] = {0};
    uint32_t pending_cursor = 0, out_cursor = 0;
    int err = 0;

    void absorb()
    {
        uint64_t in[12];
        memcpy(in, pending, 64);
        memcpy(in + 8, state, 32);
        if (zkgpu_gl_poseidon_full_host(out, in)) err = -1;
        out_cursor = 12;
        memset(pending, 0, sizeof pending);
        pending_cursor = 0;
        memcpy(state, out, 32);
    }
    void put(const uint64_t *v, uint64_t n)
    {
        for (uint64_t i = 0; i < n; i++) {
            pending[pending_cursor++] = v[i];
            out_cursor = 0;
            if (pending_cursor == 8) absorb();
        }
    }
    uint64_t get_fields1()
    {
        if (out_cursor == 0) absorb();
        uint64_t r = out[(12 - out_cursor) % 12];
        out_cursor--;
        return r;
    }
    void get_field(uint64_t o[3])
    {
        for (int i = 0; i < 3; i++) o[i] = get_fields1();
    }
    void get_permutations(uint64_t *res, uint64_t n, uint64_t nbits)
    {
        uint64_t nfields = (n * nbits - 1) / 63 + 1;
        std::vector<uint64_t> f(nfields);
        for (auto &x : f) x = get_fields1() % P;
        uint64_t cf = 0, cb = 0;
        for (uint64_t i = 0; i < n; i++) {
            uint64_t a = 0;
            for (uint64_t j = 0; j < nbits; j++) {
                if ((f[cf] >> cb) & 1) a |= 1ULL << j;
                if (++cb == 63) {
                    cb = 0;
                    cf++;
                }
            }
            res[i] = a;
        }
    }
};

// ---------------------------------------------------------------- prover
struct Prog {
    std::vector<zxp_instr> instr;
    std::vector<zxp_operand> opnd;
    uint32_t n_tmp1 = 0, n_tmp3 = 0;
    void set(const zkgpu_zxp_prog &p)
    {
        instr.assign(p.instr, p.instr + p.n_instr);
        opnd.assign(p.opnd, p.opnd + p.n_opnd);
        n_tmp1 = p.n_tmp1;
        n_tmp3 = p.n_tmp3;
    }
};

class Starks
{
public:
    zkgpu_stark_info info;
    std::vector<uint32_t> random_cols, zctx, ev, random_const, pu;
    std::vector<uint32_t> fri_steps;
    Prog step0, step1, step2, step3prev, step3, step42ns, step52ns;
    uint64_t N = 0, NE = 0;
    uint32_t eb = 0;
    zkgpu_sections S;
    std::vector<void *> allocs;
    uint64_t *nodes[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t *const_nodes = nullptr;
    uint64_t *qq1 = nullptr, *qq2 = nullptr, *cm4_n = nullptr, *lev = nullptr, *lpev = nullptr, *xdiv = nullptr, *xdivw = nullptr;
    uint64_t *fri_pol[2] = {nullptr, nullptr};
    std::vector<uint64_t *> fri_aux, fri_nodes;
    uint64_t verkey[4];
    std::vector<uint64_t> publics;
    std::vector<std::pair<std::string, double>> timers;
    // memory plan: with `dry` set, dalloc only adds up the bytes (no device)
    bool dry = false;
    uint64_t planned = 0;
    // ZKGPU_MEM_RESIDENT or ZKGPU_MEM_LEAN (include/zkgpu_stark.h)
    int mem_mode = ZKGPU_MEM_RESIDENT;
    bool lean() const { return mem_mode == ZKGPU_MEM_LEAN; }
    // lean plan: the arena (cm1_n at its start; cm1_2ns over it from stage 4),
    // cm1's stage-1 extension above cm1_n, and the n-domain columns no stage
    // writes (zeroed before their stage: the arena's regions are reused)
    uint64_t *arena = nullptr, *cm1_early = nullptr;
    std::vector<uint32_t> unwritten[5];
    bool cm1_consumed = false;
    // lean plan: cm1's last keep_cols extended columns, kept from stage 1 in
    // their own region (what the HBM left over by the plan holds) and copied
    // into place at stage 4 instead of being extended again; (n_cm1 -
    // keep_cols) is a multiple of 8 (the linear hash's chunks)
    uint64_t keep_cols = 0;
    uint64_t *keep = nullptr;
    bool lowered_lde_batch = false;  // choose_keep set the process-wide LDE batch (restored at destruction)

    // background hand-off of the next proof's cm1_n (set_cm1_async)
    // (up to two row pieces: a shard's rows wrap around the domain end)
    uint64_t *cm1_next = nullptr, *cm1_xfer[2] = {nullptr, nullptr};
    uint64_t xfer_bytes = 0;
    void *cm1_ticket[2] = {nullptr, nullptr};
    bool cm1_pending = false;

    virtual ~Starks()
    {
        if (lowered_lde_batch) zkgpu_set_lde_batch_cols(0);
        for (void *t : cm1_ticket) (void)zkgpu_load_wait(t);
        for (void *p : allocs) zkgpu_dev_free(p);
    }

    int dalloc(uint64_t **p, uint64_t elems)
    {
        if (dry) {
            planned += elems * 8;
            *p = (uint64_t *)(uintptr_t)4096;  // never dereferenced: the plan allocates nothing
            return 0;
        }
        void *v = nullptr;
        CK(zkgpu_dev_malloc(&v, elems * 8));
        allocs.push_back(v);
        // zeroed, as the reference's calloc'd memory map (prover.cpp:94-116):
        // a column no stage writes reads 0, in every proof
        CK(zkgpu_memset_dev(v, 0, elems * 8));
        *p = (uint64_t *)v;
        return 0;
    }

    // HBM a prover of this description holds at its peak: its own buffers
    // (alloc), the transient setup buffers and the library's grow-only
    // workspaces (extend_pol's column batches, the NTT scratch, the
    // expression programs' segment carries, calculateH1H2's table)
    virtual uint64_t setup_bytes() const { return 0; }
    virtual uint64_t lde_cols_max() const
    {
        return std::max({info.n_cm1, info.n_cm2, info.n_cm3, info.n_const, 1u});
    }
    virtual uint64_t prog_rows_max() const { return NE; }
    // at most this many columns per LDE batch (0: the library's default);
    // the sharded prover lowers it when its plan would not fit otherwise
    uint64_t lde_batch_cap = 0;
    int plan(uint64_t *bytes)
    {
        dry = true;
        planned = 0;
        const int rc = alloc();
        dry = false;
        if (rc) return -1;
        const uint64_t ntt_ws = std::max<uint64_t>(3, info.n_cm4) * NE * 8;  // ntt_dev scratch (workspace slot 1)
        const uint64_t lde_ws = zkgpu_lde_workspace_bytes(
            N, NE, lde_batch_cap ? std::min<uint64_t>(lde_cols_max(), lde_batch_cap) : lde_cols_max());
        const uint64_t prog_ws = 64ULL * prog_rows_max() * 8;  // <= 64 carried columns between program segments
        const uint64_t h1h2_ws = info.n_pu ? 32ULL * N : 0;    // 2N-slot table + counts + scan
        *bytes = planned + setup_bytes() + std::max(lde_ws, ntt_ws + zkgpu_lde_workspace_bytes(N, NE, 0)) + prog_ws +
                 h1h2_ws + 24ULL * N;  // + calculateZ scratch
        planned = 0;
        return 0;
    }
    // fail loudly, before any allocation, when the plan exceeds the free HBM
    int check_budget()
    {
        uint64_t need = 0, avail = 0, total = 0;
        if (plan(&need)) return -1;
        CK(zkgpu_device_memory(&avail, &total));
        if (need > avail)
            return fail("stark_create: this prover needs %.1f GB of HBM per GPU (%u-row trace, %u/%u/%u/%u committed "
                        "columns, %u constants), the device has %.1f GB free of %.1f GB",
                        need / 1e9, (unsigned)N, info.n_cm1, info.n_cm2, info.n_cm3, info.n_cm4, info.n_const,
                        avail / 1e9, total / 1e9);
        return 0;
    }

    int create(const zkgpu_stark_info *in, uint32_t mode = ZKGPU_MEM_AUTO)
    {
        if (load(in) || choose_mode(mode) || check_budget() || alloc()) return -1;
        return build_const();
    }

    // AUTO: RESIDENT when its plan fits the free HBM, else LEAN (if the
    // programs allow it; else RESIDENT, which check_budget then refuses)
    int choose_mode(uint32_t mode)
    {
        if (mode > ZKGPU_MEM_LEAN) return fail("stark_create: unknown memory plan %u", mode);
        if (mode == ZKGPU_MEM_LEAN) {
            std::string why;
            if (!lean_ok(why)) return fail("stark_create: the lean memory plan does not apply: %s", why.c_str());
            return set_mode(ZKGPU_MEM_LEAN);
        }
        mem_mode = ZKGPU_MEM_RESIDENT;
        if (mode == ZKGPU_MEM_RESIDENT) return 0;
        uint64_t need = 0, avail = 0, total = 0;
        if (plan(&need)) return -1;
        CK(zkgpu_device_memory(&avail, &total));
        std::string why;
        if (need > avail && lean_ok(why)) return set_mode(ZKGPU_MEM_LEAN);
        return 0;
    }
    int set_mode(int m, bool device = true)
    {
        mem_mode = m;
        if (m != ZKGPU_MEM_LEAN) return 0;
        find_unwritten();
        return device ? choose_keep() : 0;
    }
    // how many of cm1's extended columns the lean plan keeps from stage 1:
    // as many as the free HBM left by the plan holds (4 GB or 2 % of the
    // device spare), ZKGPU_LEAN_KEEP_COLS overriding (tests).  When not all
    // fit, LDE batches of 32 columns instead of the default 128 at 2^24 rows
    // free 19 GB of workspace for ~144 more kept columns: the LDE rate drops
    // ~1.2 % (tools/lde_batch_ab.py, profiles/r06_lde_batch_ab.json), the
    // stage-4 re-extension loses a fifth of its columns.  The batch is a
    // process-wide setting (zkgpu_set_lde_batch_cols), restored to the
    // default when this prover is destroyed.
    int choose_keep()
    {
        const uint64_t W1 = info.n_cm1;
        keep_cols = 0;
        uint64_t want = W1;
        const char *e = getenv("ZKGPU_LEAN_KEEP_COLS");
        if (e) {
            want = std::min<uint64_t>(W1, strtoull(e, nullptr, 10));
        } else {
            uint64_t avail = 0, total = 0;
            CK(zkgpu_device_memory(&avail, &total));
            const uint64_t spare = std::max<uint64_t>(4000000000ULL, total / 50);
            auto fits = [&](uint64_t cap, uint64_t &cols) {
                uint64_t need = 0;
                lde_batch_cap = cap;
                if (plan(&need)) return -1;
                cols = avail > need + spare ? std::min<uint64_t>(W1, (avail - need - spare) / (NE * 8)) : 0;
                return 0;
            };
            if (fits(0, want)) return -1;
            uint64_t want32 = 0;
            if (want < W1 && fits(32, want32)) return -1;
            if (want < W1 && want32 > want) {
                want = want32;
                zkgpu_set_lde_batch_cols(32);
                lowered_lde_batch = true;
            } else {
                lde_batch_cap = 0;
            }
        }
        const uint64_t split = W1 - want;
        keep_cols = W1 - std::min<uint64_t>(W1, (split + 7) / 8 * 8);  // (W1 - keep) a multiple of 8
        if (W1 <= 4) keep_cols = want == W1 ? W1 : 0;
        return 0;
    }

    // The lean plan needs: stage 4/5 programs that read no n-domain section
    // but the constants (their n-domain regions are gone by then), a witness
    // program that writes cm1_n only (the other n-domain regions hold cm1's
    // stage-1 extension then), and a blowup (the in-place extensions)
    bool lean_ok(std::string &why) const
    {
        if (NE < 2 * N) {
            why = "no blowup";
            return false;
        }
        const Prog *ext[2] = {&step42ns, &step52ns};
        const char *names[2] = {"step42ns", "step52ns"};
        for (int k = 0; k < 2; k++)
            for (const zxp_operand &o : ext[k]->opnd)
                if ((o.kind == ZXP_COL || o.kind == ZXP_COL3) && o.a < SEC_CONST_N) {
                    why = std::string(names[k]) + " reads an n-domain section";
                    return false;
                }
        for (const zxp_instr &i : step1.instr) {
            if (i.dst >= step1.opnd.size()) continue;
            const zxp_operand &o = step1.opnd[i.dst];
            if ((o.kind == ZXP_COL || o.kind == ZXP_COL3) && o.a != SEC_CM1_N) {
                why = "the witness program writes outside cm1_n";
                return false;
            }
        }
        return true;
    }

    // n-domain columns of tmpExp / cm2 / cm3 that no stage writes: step2,
    // calculateH1H2's h1 / h2, step3prev, calculateZ's z, step3
    void find_unwritten()
    {
        const uint32_t widths[5] = {info.n_cm1, info.n_cm2, info.n_cm3, info.n_tmp, info.n_const};
        std::vector<char> w[5];
        for (int s = 0; s < 5; s++) w[s].assign(widths[s], 0);
        for (const Prog *p : {&step2, &step3prev, &step3})
            for (const zxp_instr &i : p->instr) {
                if (i.dst >= p->opnd.size()) continue;
                const zxp_operand &o = p->opnd[i.dst];
                if ((o.kind != ZXP_COL && o.kind != ZXP_COL3) || o.a > SEC_CONST_N) continue;
                for (uint32_t c = o.b; c < o.b + (o.kind == ZXP_COL3 ? 3u : 1u) && c < widths[o.a]; c++) w[o.a][c] = 1;
            }
        for (uint32_t k = 0; k < info.n_pu; k++)
            for (uint32_t c = 0; c < pu[5 * k + 4]; c++) {
                w[SEC_CM2_N][pu[5 * k + 2] + c] = 1;
                w[SEC_CM2_N][pu[5 * k + 3] + c] = 1;
            }
        for (uint32_t z = 0; z < info.n_zctx; z++)
            for (uint32_t c = 0; c < 3; c++) w[SEC_CM3_N][zctx[3 * z + 2] + c] = 1;
        for (int s : {(int)SEC_CM2_N, (int)SEC_CM3_N, (int)SEC_TMP_N}) {
            unwritten[s].clear();
            for (uint32_t c = 0; c < widths[s]; c++)
                if (!w[s][c]) unwritten[s].push_back(c);
        }
    }
    int zero_unwritten(uint32_t s)
    {
        for (uint32_t c : unwritten[s]) CK(zkgpu_memset_dev(S.sec[s] + (uint64_t)c * N, 0, N * 8));
        return 0;
    }

    // validate the description, keep the programs, bind the device (init =
    // false: the memory plan only, no GPU)
    int load(const zkgpu_stark_info *in, bool init = true)
    {
        info = *in;
        random_cols.assign(in->random_cols, in->random_cols + in->n_random_cols);
        if (in->n_bits_ext < in->n_bits || in->n_bits_ext > 28 || in->n_fri_steps == 0 || in->n_fri_steps > 32 ||
            in->fri_steps[0] != in->n_bits_ext || in->q_deg == 0 || in->q_deg * 3 != in->n_cm4 ||
            ((uint64_t)in->q_deg << in->n_bits) > (1ULL << in->n_bits_ext) || in->l_first >= in->n_const)
            return fail("stark_create: inconsistent instance description");
        zctx.assign(in->zctx, in->zctx + 3 * in->n_zctx);
        ev.assign(in->ev, in->ev + 4 * in->n_ev);
        fri_steps.assign(in->fri_steps, in->fri_steps + in->n_fri_steps);
        if (in->n_random_const)
            random_const.assign(in->random_const, in->random_const + in->n_random_const);
        else
            for (uint32_t k = 0; k < in->n_k; k++) random_const.push_back(k);
        pu.assign(in->pu, in->pu + 5 * in->n_pu);
        for (uint32_t k = 0; k < in->n_pu; k++) {
            const uint32_t *q = &pu[5 * k];
            const uint32_t d = q[4];
            if ((d != 1 && d != 3) || q[0] + d > in->n_tmp || q[1] + d > in->n_tmp || q[2] + d > in->n_cm2 ||
                q[3] + d > in->n_cm2)
                return fail("stark_create: plookup %u out of range", k);
        }
        for (uint32_t c : random_const)
            if (c >= in->n_const) return fail("stark_create: random const column %u out of range", c);
        for (uint32_t c : random_cols)
            if (c >= in->n_cm1) return fail("stark_create: random cm1 column %u out of range", c);
        for (uint32_t z = 0; z < in->n_zctx; z++)
            if (zctx[3 * z] + 3 > in->n_tmp || zctx[3 * z + 1] + 3 > in->n_tmp || zctx[3 * z + 2] + 3 > in->n_cm3)
                return fail("stark_create: grand product %u out of range", z);
        {
            // evMap (section_2ns, col, dim, prime): starks.cpp:556-669 reads
            // pol_e[k << eb] of a 2ns section, col + dim <= its width
            const uint32_t widths_ev[5] = {in->n_cm1, in->n_cm2, in->n_cm3, in->n_cm4, in->n_const};
            for (uint32_t e = 0; e < in->n_ev; e++) {
                const uint32_t *q = &ev[4 * e];
                if (q[0] < SEC_CM1_2NS || q[0] > SEC_CONST_2NS || (q[2] != 1 && q[2] != 3) || q[3] > 1 ||
                    q[1] + q[2] > widths_ev[q[0] - SEC_CM1_2NS])
                    return fail("stark_create: evMap entry %u out of range", e);
            }
        }
        step0.set(in->step0);
        step1.set(in->step1);
        step2.set(in->step2);
        step3prev.set(in->step3prev);
        step3.set(in->step3);
        step42ns.set(in->step42ns);
        step52ns.set(in->step52ns);
        for (uint32_t si = 1; si < in->n_fri_steps; si++)
            if (in->fri_steps[si] >= in->fri_steps[si - 1] || in->fri_steps[si - 1] - in->fri_steps[si] > 5)
                return fail("stark_create: FRI steps must decrease by 1..5 bits");
        N = 1ULL << in->n_bits;
        NE = 1ULL << in->n_bits_ext;
        eb = in->n_bits_ext - in->n_bits;
        if (init) CK(zkgpu_init(-1));
        return 0;
    }

    // the n-domain sections (every prover holds them whole)
    int alloc_n()
    {
        memset(&S, 0, sizeof S);
        const zkgpu_stark_info *in = &info;
        const uint32_t widths_n[5] = {in->n_cm1, in->n_cm2, in->n_cm3, in->n_tmp, in->n_const};
        for (int s = 0; s < 5; s++) {
            if (dalloc(&S.sec[s], (uint64_t)(widths_n[s] ? widths_n[s] : 1) * N)) return -1;
            S.ld[s] = N;
            S.ncols[s] = widths_n[s];
        }
        return 0;
    }

    // stage-4/5 and FRI buffers of the whole extended domain
    int alloc_fri()
    {
        // (lean: evmap reads the quotient pieces' extended rows, no cm4_n)
        if (dalloc(&qq1, 3 * NE) || dalloc(&qq2, (uint64_t)info.n_cm4 * NE) ||
            dalloc(&cm4_n, lean() ? 1 : (uint64_t)(info.n_cm4 ? info.n_cm4 : 1) * N) || dalloc(&lev, 3 * N) ||
            dalloc(&lpev, 3 * N) || dalloc(&xdiv, 3 * NE) || dalloc(&xdivw, 3 * NE) || dalloc(&fri_pol[0], 3 * NE) ||
            dalloc(&fri_pol[1], 3 * NE))
            return -1;
        fri_aux.assign(fri_steps.size(), nullptr);
        fri_nodes.assign(fri_steps.size(), nullptr);
        for (size_t si = 1; si < fri_steps.size(); si++) {
            uint64_t len = 3ULL << fri_steps[si - 1];
            if (dalloc(&fri_aux[si], len) || dalloc(&fri_nodes[si], zkgpu_gl_merkle_num_elements(1ULL << fri_steps[si])))
                return -1;
        }
        return 0;
    }

    // The lean plan (ZKGPU_MEM_LEAN): the constants, the quotient / FRI
    // buffers and the trees are held as in the resident plan; the committed
    // sections of stages 1-3 share ONE arena of (cm1 + cm2 + cm3) extended
    // columns, laid out by their lifetimes within a proof (words, e = NE / N):
    //   [0, W1 N)            cm1_n, the proof's input (set_cm1 / witness)
    //   [W1 N, W1 N + W1 NE) stage 1: cm1_2ns, hashed into tree 1, then dead
    //   [W1 N, ...)          stages 2-3: tmpExp_n, cm2_n (in (e-1) W1 N
    //                        words; appended after the arena if larger)
    //   [W1 NE, +W2 NE)      cm2_2ns from stage 2 on
    //   [(W1+W2) NE, +W3 NE) cm3_n (bottom, stage 3), then cm3_2ns extended
    //                        in place over it
    //   [0, W1 NE)           from stage 4: cm1_2ns, extended in place over
    //                        cm1_n (whose stage-1 extension was dropped)
    // The n-domain values die after the stage-3 commit: evmap reads the
    // extended rows k << blowup with the Lagrange weights of xi / 7, as the
    // reference does (starks.cpp:308-333).
    int alloc_lean()
    {
        if (alloc_fri()) return -1;
        memset(&S, 0, sizeof S);
        const uint64_t W1 = std::max(info.n_cm1, 1u), W2 = std::max(info.n_cm2, 1u), W3 = std::max(info.n_cm3, 1u),
                       WT = std::max(info.n_tmp, 1u), WC = std::max(info.n_const, 1u);
        // resident sections: constants (both domains), cm4, q, f
        if (dalloc(&S.sec[SEC_CONST_N], WC * N) || dalloc(&S.sec[SEC_CONST_2NS], WC * NE) ||
            dalloc(&S.sec[SEC_CM4_2NS], (uint64_t)std::max(info.n_cm4, 1u) * NE) ||
            dalloc(&S.sec[SEC_Q_2NS], 3 * NE) || dalloc(&S.sec[SEC_F_2NS], 3 * NE))
            return -1;
        uint64_t words = (W1 + W2 + W3) * NE;
        const uint64_t high = W1 * N, high_words = W1 * NE - W1 * N;
        uint64_t tmp_off = high;
        if ((WT + W2) * N > high_words) {
            tmp_off = words;
            words += (WT + W2) * N;
        }
        words = std::max(words, high + (W1 - keep_cols) * NE);  // cm1's stage-1 extension (not kept)
        if (dalloc(&arena, words)) return -1;
        if (keep_cols && dalloc(&keep, keep_cols * NE)) return -1;
        S.sec[SEC_CM1_N] = arena;
        S.sec[SEC_TMP_N] = arena + tmp_off;
        S.sec[SEC_CM2_N] = arena + tmp_off + WT * N;
        S.sec[SEC_CM2_2NS] = arena + W1 * NE;
        S.sec[SEC_CM3_2NS] = arena + (W1 + W2) * NE;
        S.sec[SEC_CM3_N] = S.sec[SEC_CM3_2NS];
        cm1_early = arena + high;
        S.sec[SEC_CM1_2NS] = cm1_early;
        const uint32_t widths[SEC_COUNT] = {info.n_cm1, info.n_cm2,  info.n_cm3, info.n_tmp, info.n_const, info.n_cm1,
                                            info.n_cm2, info.n_cm3, info.n_cm4, info.n_const, 3,           3};
        for (int s = 0; s < SEC_COUNT; s++) {
            S.ld[s] = s <= SEC_CONST_N ? N : NE;
            S.ncols[s] = widths[s];
        }
        uint64_t tn = zkgpu_gl_merkle_num_elements(NE);
        for (int t = 0; t < 4; t++)
            if (dalloc(&nodes[t], tn)) return -1;
        return dalloc(&const_nodes, tn);
    }

    virtual int alloc()
    {
        if (lean()) return alloc_lean();
        if (alloc_n() || alloc_fri()) return -1;
        const zkgpu_stark_info *in = &info;
        const uint32_t widths_e[7] = {in->n_cm1, in->n_cm2, in->n_cm3, in->n_cm4, in->n_const, 3, 3};
        for (int s = 0; s < 7; s++) {
            if (dalloc(&S.sec[SEC_CM1_2NS + s], (uint64_t)(widths_e[s] ? widths_e[s] : 1) * NE)) return -1;
            S.ld[SEC_CM1_2NS + s] = NE;
            S.ncols[SEC_CM1_2NS + s] = widths_e[s];
        }
        uint64_t tn = zkgpu_gl_merkle_num_elements(NE);
        for (int t = 0; t < 4; t++)
            if (dalloc(&nodes[t], tn)) return -1;
        if (dalloc(&const_nodes, tn)) return -1;
        return 0;
    }

    // constants (setup): pseudo-random columns, L_first = [1, 0, ...], then
    // step0, on the whole n domain of S.sec[SEC_CONST_N] (ld N)
    int fill_const()
    {
        const zkgpu_stark_info *in = &info;
        CK(zkgpu_memset_dev(S.sec[SEC_CONST_N], 0, (uint64_t)in->n_const * N * 8));
        if (!random_const.empty())
            CK(zkgpu_rand_cols_dev(S.sec[SEC_CONST_N], N, random_const.data(), (uint32_t)random_const.size(), N,
                                   in->seed, 1));
        uint64_t one = 1;
        CK(zkgpu_memcpy_h2d(S.sec[SEC_CONST_N] + (uint64_t)in->l_first * N, &one, 8));
        if (!step0.instr.empty()) {
            uint64_t ch0[24] = {0}, ev0[3] = {0, 0, 0};
            if (run(step0, false, ch0, ev0, 0)) return -1;
        }
        return 0;
    }
    void init_publics()
    {
        publics.resize(info.n_publics);
        for (uint32_t k = 0; k < info.n_publics; k++) publics[k] = rand_u64(info.seed, 2, k, 0);
    }
    virtual int build_const()
    {
        if (fill_const() || commit_const()) return -1;
        init_publics();
        return 0;
    }

    int run(const Prog &p, bool ext, const uint64_t ch[24], const uint64_t *evals, uint32_t n_ev)
    {
        CK(zkgpu_zxp_eval_dev(p.instr.data(), (uint32_t)p.instr.size(), p.opnd.data(), (uint32_t)p.opnd.size(),
                              p.n_tmp1 ? p.n_tmp1 : 1, p.n_tmp3 ? p.n_tmp3 : 1, &S,
                              ext ? info.n_bits_ext : info.n_bits, ch, publics.data(), (uint32_t)publics.size(),
                              evals, n_ev, ext ? xdiv : nullptr, ext ? xdivw : nullptr, eb, ext ? 7 : 1));
        return 0;
    }

    virtual int witness()
    {
        CK(zkgpu_memset_dev(S.sec[SEC_CM1_N], 0, (uint64_t)info.n_cm1 * N * 8));
        CK(zkgpu_rand_cols_dev(S.sec[SEC_CM1_N], N, random_cols.data(), (uint32_t)random_cols.size(), N, info.seed, 0));
        uint64_t ch[24] = {0};
        uint64_t ev0[3] = {0, 0, 0};
        if (run(step1, false, ch, ev0, 0)) return -1;
        CK(zkgpu_synchronize());
        cm1_consumed = false;
        return 0;
    }

    // the executor's row-major buffer, streamed in row blocks (no full-size
    // staging copy: at the fork-9 widths cm1_n is 25-50 GB)
    virtual int set_cm1(const uint64_t *rows)
    {
        if (take_cm1_async(false)) return -1;  // a pending background load is superseded
        if (zkgpu_load_rows_dev(S.sec[SEC_CM1_N], N, rows, N, info.n_cm1, 0, 0))
            return fail("set_cm1: %s", zkgpu_last_error());
        cm1_consumed = false;
        return 0;
    }

    // cm1_n back as the executor's row-major layout (n rows x n_cm1)
    virtual int get_cm1(uint64_t *rows)
    {
        if (lean() && cm1_consumed) return fail("get_cm1: the last proof consumed the trace (lean memory plan)");
        void *tmp = nullptr;
        const uint64_t bytes = (uint64_t)info.n_cm1 * N * 8;
        CK(zkgpu_dev_malloc(&tmp, bytes ? bytes : 8));
        int rc = zkgpu_cols_to_rows_dev((uint64_t *)tmp, S.sec[SEC_CM1_N], N, N, info.n_cm1);
        if (!rc) rc = zkgpu_memcpy_d2h(rows, tmp, bytes);
        zkgpu_dev_free(tmp);
        if (rc) return fail("get_cm1: %s", zkgpu_last_error());
        return 0;
    }

    virtual int set_cm1_async(const uint64_t *rows)
    {
        if (lean())
            return fail("set_cm1_async: not offered under the lean memory plan (the proof extends cm1_n in place; "
                        "the next trace's buffer would not fit beside it); use set_cm1 between proofs");
        if (take_cm1_async(false)) return -1;
        if (cm1_next_alloc(N, 1)) return -1;
        if (zkgpu_load_rows_async(cm1_next, N, rows, N, info.n_cm1, 0, cm1_xfer[0], xfer_bytes, &cm1_ticket[0]))
            return fail("set_cm1_async: %s", zkgpu_last_error());
        cm1_pending = true;
        return 0;
    }

    // the second cm1_n buffer (ld rows per column) and `pieces` loader stages
    int cm1_next_alloc(uint64_t ld, int pieces)
    {
        if (cm1_next) return 0;
        xfer_bytes = zkgpu_load_rows_stage_bytes(ld, info.n_cm1, 0);
        if (dalloc(&cm1_next, (uint64_t)(info.n_cm1 ? info.n_cm1 : 1) * ld)) return -1;
        for (int k = 0; k < pieces; k++)
            if (dalloc(&cm1_xfer[k], std::max<uint64_t>(1, xfer_bytes / 8))) return -1;
        return 0;
    }

    // wait for a queued background load; with `use`, swap its buffer in as
    // cm1_n (every consumer reads S.sec at call time), else drop it
    int take_cm1_async(bool use)
    {
        if (!cm1_pending) return 0;
        cm1_pending = false;
        int rc = 0;
        for (void *&t : cm1_ticket) {
            const int r = zkgpu_load_wait(t);
            t = nullptr;
            rc = rc ? rc : r;
        }
        if (rc) return fail("set_cm1_async: %s", zkgpu_last_error());
        if (use) std::swap(S.sec[SEC_CM1_N], cm1_next);
        return 0;
    }

    // constant polynomials from the reference's .const file layout (N rows x
    // nConstants, ConstantPolsStarks, starks.hpp:94-116), their LDE and tree
    virtual int set_const(const uint64_t *rows)
    {
        void *tmp = nullptr;
        CK(zkgpu_dev_malloc(&tmp, (uint64_t)(info.n_const ? info.n_const : 1) * N * 8));
        int rc = zkgpu_memcpy_h2d(tmp, rows, (uint64_t)info.n_const * N * 8);
        if (!rc) rc = zkgpu_rows_to_cols_dev(S.sec[SEC_CONST_N], N, (const uint64_t *)tmp, N, info.n_const);
        if (!rc) rc = zkgpu_synchronize();
        zkgpu_dev_free(tmp);
        if (rc) return fail("set_const: %s", zkgpu_last_error());
        return commit_const();
    }

    // LDE of the constant polynomials, their tree, verkey = its root
    virtual int commit_const()
    {
        CK(zkgpu_gl_extend_pol_dev(S.sec[SEC_CONST_2NS], NE, S.sec[SEC_CONST_N], N, NE, N, info.n_const));
        CK(zkgpu_gl_merkletree_dev(const_nodes, S.sec[SEC_CONST_2NS], NE, info.n_const, NE));
        CK(zkgpu_memcpy_d2h(verkey, const_nodes + zkgpu_gl_merkle_num_elements(NE) - 4, 32));
        return 0;
    }

    int set_publics(const uint64_t *p)
    {
        for (uint32_t k = 0; k < info.n_publics; k++) publics[k] = p[k] % P;
        return 0;
    }

    uint32_t q() const { return info.n_queries; }

    uint64_t proof_len() const
    {
        uint64_t L = 16 + 3ULL * info.n_ev;
        for (size_t si = 1; si < fri_steps.size(); si++)
            L += 4 + (uint64_t)q() * (3ULL << (fri_steps[si - 1] - fri_steps[si])) + (uint64_t)q() * fri_steps[si] * 4;
        L += (uint64_t)q() * (info.n_cm1 + info.n_cm2 + info.n_cm3 + info.n_cm4 + info.n_const);
        L += 5ULL * q() * info.n_bits_ext * 4;
        L += 3ULL << fri_steps.back();
        return L;
    }

    // Stage timers (the reference's TimerStart / TimerStopAndLog) between
    // stream marks, resolved once at the end of the proof (flush_timers): a
    // stage boundary costs no device synchronisation (config-4: ~20 per
    // proof, each a dependent launch's gap); the synchronous form only when
    // the mark pool is spent
    using clk = std::chrono::steady_clock;
    clk::time_point t0;
    uint32_t t0_mark = UINT32_MAX, n_marks = 0;
    std::vector<std::pair<size_t, std::pair<uint32_t, uint32_t>>> pend_t;  // timer index, marks
    void tstart()
    {
        t0 = clk::now();
        t0_mark = UINT32_MAX;
        if (n_marks + 1 < ZKGPU_MARKS && !zkgpu_mark(n_marks)) t0_mark = n_marks++;
    }
    // ZKGPU_SYNC_STAGES=1 (debugging): a device synchronisation at every
    // stage end, so an asynchronous kernel fault is reported by the stage
    // that launched it rather than at the proof's end (flush_timers)
    bool sync_stages = [] {
        const char *e = getenv("ZKGPU_SYNC_STAGES");
        return e && atoi(e) != 0;
    }();
    int tstop(const char *name)
    {
        if (sync_stages && zkgpu_synchronize()) return fail("%s: %s", name, zkgpu_last_error());
        if (t0_mark != UINT32_MAX && n_marks < ZKGPU_MARKS && !zkgpu_mark(n_marks)) {
            pend_t.push_back({timers.size(), {t0_mark, n_marks++}});
            timers.emplace_back(name, 0.0);
            return 0;
        }
        CK(zkgpu_synchronize());
        timers.emplace_back(name, std::chrono::duration<double, std::milli>(clk::now() - t0).count());
        return 0;
    }
    // exchanges of a sharded proof: (marks, bytes sent) -> the total device
    // time inside them and that of the largest one
    std::vector<std::pair<std::pair<uint32_t, uint32_t>, uint64_t>> pend_x;
    double xchg_ms = 0, xchg_max_ms = 0;
    int flush_timers()
    {
        for (const auto &p : pend_t) {
            double ms = 0;
            CK(zkgpu_mark_elapsed(p.second.first, p.second.second, &ms));
            timers[p.first].second = ms;
        }
        pend_t.clear();
        xchg_ms = xchg_max_ms = 0;
        uint64_t big = 0;
        for (const auto &x : pend_x) {
            double ms = 0;
            CK(zkgpu_mark_elapsed(x.first.first, x.first.second, &ms));
            xchg_ms += ms;
            if (x.second >= big) {
                big = x.second;
                xchg_max_ms = ms;
            }
        }
        pend_x.clear();
        n_marks = 0;
        t0_mark = UINT32_MAX;
        return 0;
    }

    // extendPol of an n-domain section into its extended one, then its tree;
    // in place (lean plan: the section's n-domain values sit at the start of
    // its extended region) when the two pointers are equal
    int commit(int t, uint32_t sec_n, uint32_t sec_e, uint32_t ncols, Transcript &tr, uint64_t root[4],
               const char *lde_name, const char *tree_name)
    {
        tstart();
        if (S.sec[sec_e] == S.sec[sec_n])
            CK(zkgpu_gl_extend_pol_inplace_dev(S.sec[sec_e], NE, N, ncols));
        else
            CK(zkgpu_gl_extend_pol_dev(S.sec[sec_e], NE, S.sec[sec_n], N, NE, N, ncols));
        if (tstop(lde_name)) return -1;
        tstart();
        CK(zkgpu_gl_merkletree_dev(nodes[t], S.sec[sec_e], NE, ncols, NE));
        CK(zkgpu_memcpy_d2h(root, nodes[t] + zkgpu_gl_merkle_num_elements(NE) - 4, 32));
        if (tstop(tree_name)) return -1;
        tr.put(root, 4);
        return 0;
    }

    // lean plan, stage 1: cm1's extension into the scratch above cm1_n
    // (columns [0, split), hashed and dropped) and into `keep` (the rest,
    // kept for stage 4), one tree over both regions
    int commit_cm1_lean(Transcript &tr, uint64_t root[4])
    {
        const uint64_t W1 = info.n_cm1, split = W1 - keep_cols;
        S.sec[SEC_CM1_2NS] = cm1_early;
        tstart();
        if (split) CK(zkgpu_gl_extend_pol_dev(cm1_early, NE, arena, N, NE, N, split));
        if (keep_cols) CK(zkgpu_gl_extend_pol_dev(keep, NE, arena + split * N, N, NE, N, keep_cols));
        if (tstop("STARK_STEP_1_LDE")) return -1;
        tstart();
        if (!keep_cols)
            CK(zkgpu_gl_merkletree_dev(nodes[0], cm1_early, NE, W1, NE));
        else if (!split)
            CK(zkgpu_gl_merkletree_dev(nodes[0], keep, NE, W1, NE));
        else
            CK(zkgpu_gl_merkletree2_dev(nodes[0], cm1_early, keep, NE, split, W1, NE));
        CK(zkgpu_memcpy_d2h(root, nodes[0] + zkgpu_gl_merkle_num_elements(NE) - 4, 32));
        if (tstop("STARK_STEP_1_MERKLETREE")) return -1;
        tr.put(root, 4);
        return 0;
    }

    // the proof of the current cm1_n; a trace queued by set_cm1_async (loaded
    // meanwhile) becomes cm1_n when it returns
    virtual int prove(uint64_t *out)
    {
        if (lean() && cm1_consumed)
            return fail("stark_prove: the previous proof consumed the trace (lean memory plan: cm1_n is extended in "
                        "place); load the next one with set_cm1 or witness first");
        const int rc = prove_body(out);
        const int rc2 = take_cm1_async(true);
        return rc ? rc : rc2;
    }

    int prove_body(uint64_t *out)
    {
        timers.clear();
        pend_t.clear();
        pend_x.clear();
        n_marks = 0;
        auto tall = clk::now();
        Transcript tr;
        tr.put(verkey, 4);
        tr.put(publics.data(), publics.size());
        uint64_t ch[24] = {0};
        uint64_t roots[4][4];
        std::vector<uint64_t> evals(3 * info.n_ev);
        // STAGE 1 (starks.cpp:49-63)
        if (lean()) {
            if (commit_cm1_lean(tr, roots[0])) return -1;
        } else if (commit(0, SEC_CM1_N, SEC_CM1_2NS, info.n_cm1, tr, roots[0], "STARK_STEP_1_LDE",
                          "STARK_STEP_1_MERKLETREE")) {
            return -1;
        }
        // lean: the regions of tmpExp_n / cm2_n / cm3_n held other sections;
        // the columns no stage writes read 0, as under the resident plan
        if (lean() && (zero_unwritten(SEC_TMP_N) || zero_unwritten(SEC_CM2_N) || zero_unwritten(SEC_CM3_N)))
            return -1;
        // STAGE 2 (:65-144)
        tr.get_field(ch + 0);
        tr.get_field(ch + 3);
        tstart();
        if (run(step2, false, ch, evals.data(), 0)) return -1;
        if (tstop("STARK_STEP_2_CALCULATE_EXPS")) return -1;
        if (info.n_pu) {
            tstart();
            if (h1h2_all()) return -1;
            if (tstop("STARK_STEP_2_CALCULATEH1H2")) return -1;
        }
        if (commit(1, SEC_CM2_N, SEC_CM2_2NS, info.n_cm2, tr, roots[1], "STARK_STEP_2_LDE", "STARK_STEP_2_MERKLETREE"))
            return -1;
        // STAGE 3 (:146-224)
        tr.get_field(ch + 6);
        tr.get_field(ch + 9);
        tstart();
        if (run(step3prev, false, ch, evals.data(), 0)) return -1;
        if (tstop("STARK_STEP_3_CALCULATE_EXPS")) return -1;
        tstart();
        if (z_all()) return -1;
        if (tstop("STARK_STEP_3_CALCULATE_Z")) return -1;
        // step3: post-Z expressions (starks.cpp:193-208)
        if (!step3.instr.empty()) {
            tstart();
            if (run(step3, false, ch, evals.data(), 0)) return -1;
            if (tstop("STARK_STEP_3_CALCULATE_EXPS_2")) return -1;
        }
        if (commit(2, SEC_CM3_N, SEC_CM3_2NS, info.n_cm3, tr, roots[2], "STARK_STEP_3_LDE", "STARK_STEP_3_MERKLETREE"))
            return -1;
        // STAGE 4 (:226-296)
        tr.get_field(ch + 12);
        if (lean()) {
            // cm1_2ns again, over cm1_n (tmpExp_n / cm2_n above it are dead):
            // the columns not kept extended in place, the kept ones copied
            tstart();
            cm1_consumed = true;
            const uint64_t split = info.n_cm1 - keep_cols;
            if (split) CK(zkgpu_gl_extend_pol_inplace_dev(arena, NE, N, split));
            if (keep_cols) CK(zkgpu_memcpy_d2d(arena + split * NE, keep, keep_cols * NE * 8));
            S.sec[SEC_CM1_2NS] = arena;
            if (tstop("STARK_STEP_4_CM1_LDE")) return -1;
        }
        tstart();
        if (run(step42ns, true, ch, evals.data(), 0)) return -1;
        if (tstop("STARK_STEP_4_CALCULATE_EXPS_2NS")) return -1;
        tstart();
        if (quotient_pieces(S.sec[SEC_Q_2NS], S.sec[SEC_CM4_2NS])) return -1;
        if (tstop("STARK_STEP_4_CALCULATE_EXPS_2NS_INTT_NTT")) return -1;
        tstart();
        CK(zkgpu_gl_merkletree_dev(nodes[3], S.sec[SEC_CM4_2NS], NE, info.n_cm4, NE));
        CK(zkgpu_memcpy_d2h(roots[3], nodes[3] + zkgpu_gl_merkle_num_elements(NE) - 4, 32));
        if (tstop("STARK_STEP_4_MERKLETREE")) return -1;
        tr.put(roots[3], 4);
        // STAGE 5 (:298-392)
        tstart();
        uint64_t *xi = ch + 21;
        tr.get_field(xi);
        // Starks::evmap (starks.cpp:308-333,556-669) interpolates every
        // polynomial from its extension rows k << eb, the coset points
        // 7 w_N^k, with L = INTT((xi/7)^i).  The same values pol(xi) come
        // from the n-domain rows (points w_N^k) with L = INTT(xi^i): the
        // polynomial of degree < N is the same, the field sums are exact, and
        // contiguous n-domain columns read half the lines of the strided
        // extension rows.
        if (lean()) {
            // the extended rows k << eb are the points 7 w_N^k: the weights of
            // xi / 7 (starks.cpp:316-322)
            const uint64_t i7 = inv(7), xs[3] = {mul(xi[0], i7), mul(xi[1], i7), mul(xi[2], i7)};
            if (lagrange_xi(xs, 0, N)) return -1;
        } else if (lagrange_xi(xi, 0, N)) {
            return -1;
        }
        if (tstop("STARK_STEP_5_LEv_LpEv")) return -1;
        tstart();
        if (evmap_rows(0, N, evals.data())) return -1;
        if (tstop("STARK_STEP_5_EVMAP")) return -1;
        tr.put(evals.data(), evals.size());
        tr.get_field(ch + 15);
        tr.get_field(ch + 18);
        tstart();
        CK(zkgpu_xdivxsub_dev(xdiv, xdivw, xi, info.n_bits, info.n_bits_ext));
        if (tstop("STARK_STEP_5_XDIVXSUB")) return -1;
        tstart();
        if (run(step52ns, true, ch, evals.data(), info.n_ev)) return -1;
        CK(zkgpu_cols3_to_interleaved_dev(fri_pol[0], S.sec[SEC_F_2NS], NE, NE));
        if (tstop("STARK_STEP_5_CALCULATE_EXPS")) return -1;
        return fri_and_queries(tr, &roots[0][0], evals, out, tall);
    }

    // calculateH1H2 of every plookup (starks.cpp:104-127), n domain
    virtual int h1h2_all()
    {
        for (uint32_t k = 0; k < info.n_pu; k++) {
            const uint32_t *q = &pu[5 * k];
            uint64_t miss = 0;
            const int rc = zkgpu_h1h2_dev(S.sec[SEC_CM2_N] + (uint64_t)q[2] * N, N,
                                          S.sec[SEC_CM2_N] + (uint64_t)q[3] * N, N,
                                          S.sec[SEC_TMP_N] + (uint64_t)q[0] * N, N,
                                          S.sec[SEC_TMP_N] + (uint64_t)q[1] * N, N, N, q[4], &miss);
            if (rc) {
                if (miss != ~0ULL)
                    return fail("Polinomial::calculateH1H2() Number not included: w=%llu plookup_number=%u",
                                (unsigned long long)miss, k);
                return fail("calculateH1H2: %s", zkgpu_last_error());
            }
        }
        return 0;
    }

    // calculateZ of every grand product (starks.cpp:165-189), n domain
    virtual int z_all()
    {
        std::vector<zkgpu_z_req> req(info.n_zctx);
        for (uint32_t z = 0; z < info.n_zctx; z++)
            req[z] = {S.sec[SEC_CM3_N] + (uint64_t)zctx[3 * z + 2] * N, N, S.sec[SEC_TMP_N] + (uint64_t)zctx[3 * z] * N, N,
                      S.sec[SEC_TMP_N] + (uint64_t)zctx[3 * z + 1] * N, N};
        std::vector<int> closes(info.n_zctx + 1, 0);
        CK(zkgpu_calculate_z_many_dev(req.data(), info.n_zctx, N, closes.data()));
        for (uint32_t z = 0; z < info.n_zctx; z++)
            if (!closes[z]) return fail("calculateZ: grand product %u does not close", z);
        return 0;
    }

    // LEv / LpEv: the n-domain Lagrange weights of xi and w xi (see prove),
    // rows [row0, row0 + nrows) in closed form (zkgpu_lagrange_xi_rows_dev);
    // the whole domain by interpolation when xi lies in the base field
    int lagrange_xi(const uint64_t xi[3], uint64_t row0, uint64_t nrows)
    {
        if (xi[1] % P || xi[2] % P) {
            CK(zkgpu_lagrange_xi_rows_dev(lev + row0, lpev + row0, N, xi, info.n_bits, row0, nrows));
            return 0;
        }
        uint64_t wN = w_of(info.n_bits);
        uint64_t xis[3], wxis[3];
        for (int k = 0; k < 3; k++) {
            xis[k] = xi[k] % P;
            wxis[k] = mul(xi[k], wN);
        }
        CK(zkgpu_ext_powers_dev(lev, N, xis, N));
        CK(zkgpu_ext_powers_dev(lpev, N, wxis, N));
        CK(zkgpu_gl_ntt_dev(lev, N, lev, N, N, 3, 1));
        CK(zkgpu_gl_ntt_dev(lpev, N, lpev, N, N, 3, 1));
        return 0;
    }

    // starks.cpp:255-296: q (NE x 3, column-major, ld NE) -> INTT -> split
    // into q_deg pieces -> NTT on the coset -> cm4 (n_cm4 x NE); the pieces
    // on the n domain too (cm4_n, for evmap)
    int quotient_pieces(const uint64_t *q, uint64_t *cm4)
    {
        CK(zkgpu_gl_ntt_dev(qq1, NE, q, NE, NE, 3, 1));
        CK(zkgpu_memset_dev(qq2, 0, (uint64_t)info.n_cm4 * NE * 8));
        uint64_t shift_in = pw(inv(7), N);
        CK(zkgpu_qsplit_dev(qq2, NE, qq1, NE, N, info.q_deg, shift_in));
        CK(zkgpu_gl_ntt_dev(cm4, NE, qq2, NE, NE, info.n_cm4, 0));
        if (lean()) return 0;  // evmap reads the pieces' extended rows
        // the quotient pieces on the n-domain too (for evmap below): qq2 holds
        // coset-scaled coefficients c_k 7^k (k < N, the rest zero); plain
        // coefficients c_k = qq2_k 7^-k, then NTT_N -> q_p(w_N^j)
        for (uint32_t c = 0; c < info.n_cm4; c++)
            CK(zkgpu_memcpy_d2d(cm4_n + (uint64_t)c * N, qq2 + (uint64_t)c * NE, N * 8));
        CK(zkgpu_scale_by_powers_dev(cm4_n, N, info.n_cm4, N, inv(7)));
        CK(zkgpu_gl_ntt_dev(cm4_n, N, cm4_n, N, N, info.n_cm4, 0));
        return 0;
    }

    // the n-domain values of an evMap entry's polynomial (section_2ns ev_sec,
    // column col) from global row `row` on, and their leading dimension
    virtual const uint64_t *ncol(uint32_t ev_sec, uint32_t col, uint64_t row, uint64_t &ld) const
    {
        ld = N;
        if (ev_sec == SEC_CM4_2NS) return cm4_n + (uint64_t)col * N + row;
        const uint32_t s = ev_sec == SEC_CONST_2NS ? (uint32_t)SEC_CONST_N : ev_sec - SEC_CM1_2NS + SEC_CM1_N;
        return S.sec[s] + (uint64_t)col * N + row;
    }

    // Starks::evmap over n-domain rows [k0, k0 + nrows) (starks.cpp:556-669;
    // the row sum is linear, so row blocks give partial sums)
    int evmap_rows(uint64_t k0, uint64_t nrows, uint64_t *evals_out)
    {
        std::vector<const uint64_t *> cols(info.n_ev);
        std::vector<uint64_t> lds(info.n_ev);
        std::vector<uint32_t> dims(info.n_ev), primes(info.n_ev);
        for (uint32_t e = 0; e < info.n_ev; e++) {
            if (lean()) {  // the extended rows k << eb (the n-domain values are gone)
                lds[e] = NE;
                cols[e] = S.sec[ev[4 * e]] + (uint64_t)ev[4 * e + 1] * NE + (k0 << eb);
            } else {
                cols[e] = ncol(ev[4 * e], ev[4 * e + 1], k0, lds[e]);
            }
            dims[e] = ev[4 * e + 2];
            primes[e] = ev[4 * e + 3];
        }
        CK(zkgpu_evmap_dev(evals_out, cols.data(), lds.data(), dims.data(), primes.data(), info.n_ev, lev + k0,
                           lpev + k0, N, nrows, lean() ? eb : 0));
        return 0;
    }

    // FRIProve::prove + queries (friProve.cpp:5-232) once fri_pol[0] holds the
    // FRI polynomial; s0 openings through open_s0
    int fri_and_queries(Transcript &tr, const uint64_t *roots, const std::vector<uint64_t> &evals, uint64_t *out,
                        clk::time_point tall)
    {
        tstart();
        uint64_t *w = out;
        memcpy(w, roots, 16 * 8);
        w += 16;
        memcpy(w, evals.data(), evals.size() * 8);
        w += evals.size();
        uint32_t pol_bits = info.n_bits_ext;
        uint64_t shift_inv = inv(7);
        int cur = 0;
        std::vector<uint64_t> fri_roots(4 * fri_steps.size(), 0);
        std::vector<uint64_t> final_pol(3ULL << fri_steps.back());
        for (size_t si = 0; si < fri_steps.size(); si++) {
            uint32_t red = pol_bits - fri_steps[si];
            uint64_t sx[3];
            tr.get_field(sx);
            if (si > 0) {
                if (fri_fold_step(si, fri_pol[cur ^ 1], fri_pol[cur], pol_bits, fri_steps[si], sx, shift_inv)) return -1;
                cur ^= 1;
            }
            if (si < fri_steps.size() - 1) {
                uint32_t nb = fri_steps[si + 1];
                uint64_t ngroups = 1ULL << nb;
                uint64_t width = (3ULL << fri_steps[si]) / ngroups;
                // (layer 0 of a prover that keeps f in row blocks: no whole
                // fri_pol[0] exists, the override reads the blocks)
                const uint64_t *pol = si == 0 && !fri_pol0_filled() ? nullptr : fri_pol[cur];
                if (fri_transpose_layer(si, fri_aux[si + 1], pol, 1ULL << fri_steps[si], nb)) return -1;
                if (fri_commit(si + 1, ngroups, width, &fri_roots[4 * (si + 1)])) return -1;
                tr.put(&fri_roots[4 * (si + 1)], 4);
            } else {
                CK(zkgpu_memcpy_d2h(final_pol.data(), fri_pol[cur], final_pol.size() * 8));
                tr.put(final_pol.data(), final_pol.size());
            }
            pol_bits = fri_steps[si];
            for (uint32_t j = 0; j < red; j++) shift_inv = mul(shift_inv, shift_inv);
        }
        if (tstop("STARK_STEP_FRI_FOLDS")) return -1;
        tstart();
        std::vector<uint64_t> ys(q());
        tr.get_permutations(ys.data(), q(), fri_steps[0]);
        pend.clear();
        pend_idx.clear();
        // FRI layers si >= 1: root, vals, siblings
        std::vector<uint64_t> yq = ys;
        for (size_t si = 0; si < fri_steps.size(); si++) {
            if (si > 0) {  // root, then the openings written in place (at flush_opens at the latest)
                uint64_t ngroups = 1ULL << fri_steps[si];
                uint64_t width = (3ULL << fri_steps[si - 1]) / ngroups;
                memcpy(w, &fri_roots[4 * si], 32);
                w += 4;
                uint64_t *vals = w, *sibs = w + q() * width;
                w = sibs + (uint64_t)q() * fri_steps[si] * 4;
                if (fri_open(si, ngroups, width, yq, vals, sibs)) return -1;
            }
            if (si < fri_steps.size() - 1)
                for (auto &y : yq) y %= (1ULL << fri_steps[si + 1]);
        }
        if (open_s0(ys, w) || flush_opens()) return -1;
        memcpy(w, final_pol.data(), final_pol.size() * 8);
        w += final_pol.size();
        if (tstop("STARK_STEP_FRI_QUERIES") || flush_timers()) return -1;
        if (tr.err) return fail("transcript hashing failed: %s", zkgpu_last_error());
        if ((uint64_t)(w - out) != proof_len()) return fail("proof length mismatch");
        timers.emplace_back("STARK_TOTAL", std::chrono::duration<double, std::milli>(clk::now() - tall).count());
        return 0;
    }

    // fold step si: 2^pol_bits -> 2^out_bits elements (friProve.cpp:44-108)
    virtual int fri_fold_step(size_t si, uint64_t *dst, const uint64_t *src, uint32_t pol_bits, uint32_t out_bits,
                              const uint64_t sx[3], uint64_t shift_inv)
    {
        (void)si;
        CK(zkgpu_fri_fold_dev(dst, src, pol_bits, out_bits, sx, shift_inv));
        return 0;
    }
    // whether fri_pol[0] holds the whole FRI polynomial when the FRI loop
    // starts (the row-sharded prover keeps it in row blocks instead)
    virtual bool fri_pol0_filled() const { return true; }
    // layer si + 1's tree rows: getTransposed of the 2^pol_bits-element
    // polynomial of step si into 2^nb groups (friProve.cpp:111-121)
    virtual int fri_transpose_layer(size_t si, uint64_t *aux, const uint64_t *pol, uint64_t degree, uint32_t nb)
    {
        (void)si;
        CK(zkgpu_fri_transpose_dev(aux, pol, degree, nb));
        return 0;
    }
    // FRI layer si's tree over its ngroups x width row-major groups (friProve.cpp:125-133)
    virtual int fri_commit(size_t si, uint64_t ngroups, uint64_t width, uint64_t root[4])
    {
        CK(zkgpu_gl_merkletree_rows_dev(fri_nodes[si], fri_aux[si], width, ngroups));
        CK(zkgpu_memcpy_d2h(root, fri_nodes[si] + zkgpu_gl_merkle_num_elements(ngroups) - 4, 32));
        return 0;
    }
    // its openings at groups yq (vals q x width, siblings q x log2(ngroups) x 4)
    // (queued: written by flush_opens, all of a proof's openings in one round trip)
    virtual int fri_open(size_t si, uint64_t ngroups, uint64_t width, const std::vector<uint64_t> &yq, uint64_t *vals,
                         uint64_t *sibs)
    {
        pend_idx.emplace_back(yq);
        pend.push_back({vals, sibs, fri_nodes[si], fri_aux[si], 0, width, ngroups, pend_idx.back().data(), q(), 1});
        return 0;
    }

    // s0: the 4 stage trees + the constant tree at the original indices
    // (queued like fri_open): vals of the 5 trees, then their siblings
    virtual int open_s0(const std::vector<uint64_t> &ys, uint64_t *&w)
    {
        const uint32_t secs[5] = {SEC_CM1_2NS, SEC_CM2_2NS, SEC_CM3_2NS, SEC_CM4_2NS, SEC_CONST_2NS};
        const uint32_t widths[5] = {info.n_cm1, info.n_cm2, info.n_cm3, info.n_cm4, info.n_const};
        uint64_t *trees[5] = {nodes[0], nodes[1], nodes[2], nodes[3], const_nodes};
        uint64_t *sib = w;
        for (int t = 0; t < 5; t++) sib += (uint64_t)q() * widths[t];
        pend_idx.emplace_back(ys);
        for (int t = 0; t < 5; t++) {
            pend.push_back({w, sib, trees[t], S.sec[secs[t]], NE, widths[t], NE, pend_idx.back().data(), q(), 0});
            w += (uint64_t)q() * widths[t];
            sib += (uint64_t)q() * info.n_bits_ext * 4;
        }
        w = sib;
        return 0;
    }

    // the queued openings (fri_open / open_s0 of this class)
    std::vector<zkgpu_open_req> pend;
    std::vector<std::vector<uint64_t>> pend_idx;
    int flush_opens()
    {
        const int rc = pend.empty() ? 0 : zkgpu_gl_merkle_open_many(pend.data(), (uint32_t)pend.size());
        pend.clear();
        pend_idx.clear();
        CK(rc);
        return 0;
    }
};

#include "sharded_starks.hpp"

}  // namespace zkgpu_host

#include "comm_host.hpp"
#include "comm_rccl.hpp"

using zkgpu_host::ShardedStarks;
using zkgpu_host::Starks;

extern "C" {

const char *zkgpu_stark_last_error(void) { return zkgpu_host::g_err; }

int zkgpu_stark_create_ex(void **handle, const zkgpu_stark_info *info, uint32_t memory_plan)
{
    Starks *s = new Starks();
    if (s->create(info, memory_plan)) {
        delete s;
        *handle = nullptr;
        return -1;
    }
    *handle = s;
    return 0;
}

int zkgpu_stark_create(void **handle, const zkgpu_stark_info *info)
{
    return zkgpu_stark_create_ex(handle, info, ZKGPU_MEM_AUTO);
}

int zkgpu_stark_memory_mode(void *h) { return ((Starks *)h)->mem_mode; }

int zkgpu_stark_witness(void *h) { return ((Starks *)h)->witness(); }
int zkgpu_stark_set_cm1(void *h, const uint64_t *rows) { return ((Starks *)h)->set_cm1(rows); }
int zkgpu_stark_set_cm1_async(void *h, const uint64_t *rows) { return ((Starks *)h)->set_cm1_async(rows); }
int zkgpu_stark_get_cm1(void *h, uint64_t *rows) { return ((Starks *)h)->get_cm1(rows); }
int zkgpu_stark_set_const(void *h, const uint64_t *rows) { return ((Starks *)h)->set_const(rows); }
int zkgpu_stark_set_publics(void *h, const uint64_t *publics) { return ((Starks *)h)->set_publics(publics); }
uint64_t zkgpu_stark_proof_len(void *h) { return ((Starks *)h)->proof_len(); }
int zkgpu_stark_prove(void *h, uint64_t *out) { return ((Starks *)h)->prove(out); }
int zkgpu_stark_verkey(void *h, uint64_t out[4])
{
    memcpy(out, ((Starks *)h)->verkey, 32);
    return 0;
}
int zkgpu_stark_publics(void *h, uint64_t *out)
{
    Starks *s = (Starks *)h;
    memcpy(out, s->publics.data(), s->publics.size() * 8);
    return (int)s->publics.size();
}
int zkgpu_stark_timers(void *h, char *names_buf, uint64_t names_len, double *ms, uint32_t max)
{
    Starks *s = (Starks *)h;
    std::string names;
    uint32_t n = 0;
    for (auto &t : s->timers) {
        if (n >= max) break;
        names += t.first + "\n";
        ms[n++] = t.second;
    }
    if (names_len) {
        size_t c = names.size() < names_len - 1 ? names.size() : names_len - 1;
        memcpy(names_buf, names.data(), c);
        names_buf[c] = 0;
    }
    return (int)n;
}
void zkgpu_stark_destroy(void *h) { delete (Starks *)h; }

// the prover's own Transcript class behind the reference's Transcript surface
struct zkgpu_transcript {
    zkgpu_host::Transcript t;
};
zkgpu_transcript *zkgpu_transcript_create(void) { return new zkgpu_transcript(); }
void zkgpu_transcript_destroy(zkgpu_transcript *t) { delete t; }
int zkgpu_transcript_put(zkgpu_transcript *t, const uint64_t *in, uint64_t n)
{
    if (!t || (n && !in)) return zkgpu_host::fail("transcript_put: null argument");
    t->t.put(in, n);
    return t->t.err ? zkgpu_host::fail("transcript_put: host permutation failed") : 0;
}
int zkgpu_transcript_get_fields1(zkgpu_transcript *t, uint64_t *out)
{
    if (!t || !out) return zkgpu_host::fail("transcript_get_fields1: null argument");
    *out = t->t.get_fields1();
    return t->t.err ? zkgpu_host::fail("transcript_get_fields1: host permutation failed") : 0;
}
int zkgpu_transcript_get_field(zkgpu_transcript *t, uint64_t out[3])
{
    if (!t || !out) return zkgpu_host::fail("transcript_get_field: null argument");
    t->t.get_field(out);
    return t->t.err ? zkgpu_host::fail("transcript_get_field: host permutation failed") : 0;
}
int zkgpu_transcript_get_permutations(zkgpu_transcript *t, uint64_t *res, uint64_t n, uint64_t nbits)
{
    if (!t || (n && !res)) return zkgpu_host::fail("transcript_get_permutations: null argument");
    if (nbits == 0 || nbits > 63) return zkgpu_host::fail("transcript_get_permutations: nbits %lu not in [1, 63]", (unsigned long)nbits);
    if (n == 0) return 0;
    t->t.get_permutations(res, n, nbits);
    return t->t.err ? zkgpu_host::fail("transcript_get_permutations: host permutation failed") : 0;
}

int zkgpu_stark_create_sharded(void **handle, const zkgpu_stark_info *info, const zkgpu_comm *comm)
{
    *handle = nullptr;
    if (!comm) return zkgpu_host::fail("stark_create_sharded: no communicator");
    ShardedStarks *s = new ShardedStarks();
    if (s->create_sharded(info, comm)) {
        delete s;
        return -1;
    }
    *handle = s;
    return 0;
}

int zkgpu_stark_memory_plan(const zkgpu_stark_info *info, uint32_t world, uint64_t *bytes_per_gpu)
{
    if (!info || !bytes_per_gpu) return zkgpu_host::fail("stark_memory_plan: null argument");
    *bytes_per_gpu = 0;
    if (world == 0) {
        Starks s;
        if (s.load(info, false)) return -1;
        return s.plan(bytes_per_gpu);
    }
    ShardedStarks s;
    if (s.shape(info, world, 0, false)) return -1;
    return s.plan(bytes_per_gpu);
}

int zkgpu_stark_memory_plan_ex(const zkgpu_stark_info *info, uint32_t memory_plan, uint64_t *bytes)
{
    if (!info || !bytes) return zkgpu_host::fail("stark_memory_plan_ex: null argument");
    *bytes = 0;
    if (memory_plan > ZKGPU_MEM_LEAN) return zkgpu_host::fail("stark_memory_plan_ex: unknown plan %u", memory_plan);
    Starks s;
    if (s.load(info, false)) return -1;
    if (memory_plan == ZKGPU_MEM_LEAN) {
        std::string why;
        if (!s.lean_ok(why)) return zkgpu_host::fail("stark_memory_plan_ex: the lean plan does not apply: %s", why.c_str());
        s.set_mode(ZKGPU_MEM_LEAN, false);  // (no device: no kept columns)
    }
    return s.plan(bytes);
}

int zkgpu_comm_rccl_unique_id(uint8_t id[128])
{
    using zkgpu_host::g_rccl;
    if (g_rccl.load()) return -1;
    ncclUniqueId u;
    ncclResult_t r = g_rccl.get_unique_id(&u);
    if (r != ncclSuccess) return zkgpu_host::fail("ncclGetUniqueId: %s", g_rccl.error_string(r));
    static_assert(sizeof u == 128, "ncclUniqueId size");
    memcpy(id, &u, 128);
    return 0;
}

int zkgpu_comm_rccl_create(zkgpu_comm *comm, const uint8_t id[128], uint32_t world, uint32_t rank)
{
    using zkgpu_host::g_rccl;
    memset(comm, 0, sizeof *comm);
    if (g_rccl.load()) return -1;
    if (zkgpu_init(-1)) return zkgpu_host::fail("zkgpu_comm_rccl_create: %s", zkgpu_last_error());
    ncclUniqueId u;
    memcpy(&u, id, 128);
    auto *ctx = new zkgpu_host::RcclCtx();
    ncclResult_t r = g_rccl.comm_init_rank(&ctx->comm, (int)world, u, (int)rank);
    if (r != ncclSuccess) {
        delete ctx;
        return zkgpu_host::fail("ncclCommInitRank(world %u, rank %u): %s", world, rank, g_rccl.error_string(r));
    }
    comm->rank = rank;
    comm->world = world;
    comm->ctx = ctx;
    comm->exchange = zkgpu_host::rccl_exchange;
    comm->abort = zkgpu_host::rccl_abort;
    return 0;
}

int zkgpu_comm_host_create(zkgpu_comm *comm, const char *name, uint32_t world, uint32_t rank, uint64_t capacity)
{
    return zkgpu_host::host_comm_create(comm, name, world, rank, capacity);
}

void zkgpu_comm_host_destroy(zkgpu_comm *comm) { zkgpu_host::host_comm_destroy(comm); }

void zkgpu_comm_rccl_destroy(zkgpu_comm *comm)
{
    if (!comm || !comm->ctx) return;
    auto *ctx = (zkgpu_host::RcclCtx *)comm->ctx;
    if (ctx->comm && !ctx->aborted && zkgpu_host::g_rccl.comm_destroy) zkgpu_host::g_rccl.comm_destroy(ctx->comm);
    if (ctx->done) (void)hipEventDestroy(ctx->done);
    delete ctx;
    comm->ctx = nullptr;
    comm->exchange = nullptr;
    comm->abort = nullptr;
}

}  // extern "C"
