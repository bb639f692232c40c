// Segmented expression programs (see zxp_segment.hpp).
//
// The zkEVM's constraint quotient (step42ns, zkevm.chelpers.step42ns.parser.cpp:
// 11-793, 18.5 K ops per row) compiles to one straight-line kernel of ~7 K
// compiled instructions: 5 MB of code, 322 VGPRs (one wave per SIMD) and
// ~20 minutes of hiprtc.  Cut into segments, every kernel is a fraction of
// that: each compiles on its own (in parallel), holds only its own stretch of
// the program in registers and in the instruction cache, and the values that
// cross a cut travel through scratch columns.  The combination of the
// constraints is linear (the alpha Horner chain is a sum of DOTs), so a cut
// anywhere is exact: the carried values are field elements, stored canonical.
#include "zxp_segment.hpp"

#include <algorithm>
#include <cstring>

#include "../../include/zkgpu.h"

namespace zk {
int set_error(int code, const char *fmt, ...);  // api.hip
}

namespace zk {

namespace {

uint32_t opnd_dim(const zxp_operand &o)
{
    switch (o.kind) {
    case ZXP_TMP3:
    case ZXP_COL3:
    case ZXP_CHAL:
    case ZXP_EVAL:
    case ZXP_XDIV:
    case ZXP_XDIVW: return 3;
    case ZXP_IMM: return o.b == 3 ? 3 : 1;
    default: return 1;
    }
}

bool is_tmp(const zxp_operand &o) { return o.kind == ZXP_TMP1 || o.kind == ZXP_TMP3; }

}  // namespace

uint32_t zxp_instr_cost(const zxp_compiled &cp, uint32_t k)
{
    const zxp_instr &I = cp.instr[k];
    if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
        uint32_t n = 0;
        for (uint32_t t = I.a; t < I.a + I.b; t++) n += cp.term[t].src != ZXP_TERM_ONE;
        return I.op == ZXP_DOT3 ? 30 + 20 * n : 10 + 7 * n;
    }
    if (I.op == ZXP_COPY) return 1;
    const uint32_t da = opnd_dim(cp.opnd[I.a]), db = opnd_dim(cp.opnd[I.b]);
    if (I.op == ZXP_MUL) return da == 3 && db == 3 ? 160 : (da == 3 || db == 3) ? 66 : 22;
    return 7 * std::max(da, db);
}

int zxp_segment(const zxp_compiled &cp, uint32_t n_seg, std::vector<ZxpSegment> &out, uint32_t &n_scratch)
{
    out.clear();
    n_scratch = 0;
    const uint32_t n = cp.n_instr, n_op = cp.n_opnd;
    if (n_seg < 2 || n < 2 * n_seg) n_seg = std::max<uint32_t>(1, std::min<uint32_t>(n_seg, n / 2));
    // SSA temporaries: one definition each (zkgpu_zxp_compile), then reads
    std::vector<int64_t> def(n_op, -1), last(n_op, -1);
    auto reads = [&](uint32_t k, auto &&f) {
        const zxp_instr &I = cp.instr[k];
        if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
            for (uint32_t t = I.a; t < I.a + I.b; t++)
                if (cp.term[t].src != ZXP_TERM_ONE) f(cp.term[t].src);
        } else {
            f(I.a);
            if (I.op != ZXP_COPY) f(I.b);
        }
    };
    for (uint32_t k = 0; k < n; k++) {
        const zxp_instr &I = cp.instr[k];
        if (I.dst >= n_op) return set_error(ZKGPU_ERR_ARG, "zxp segment: instruction %u destination", k);
        bool bad = false;
        reads(k, [&](uint32_t o) {
            if (o >= n_op) {
                bad = true;
                return;
            }
            if (is_tmp(cp.opnd[o])) {
                if (def[o] < 0) bad = true;  // read before its definition
                last[o] = k;
            }
        });
        if (bad) return set_error(ZKGPU_ERR_ARG, "zxp segment: instruction %u reads an undefined value", k);
        if (is_tmp(cp.opnd[I.dst])) {
            if (def[I.dst] >= 0) return set_error(ZKGPU_ERR_ARG, "zxp segment: temporary %u defined twice", I.dst);
            def[I.dst] = k;
        }
    }
    // words live across the boundary before instruction j
    std::vector<int64_t> delta((size_t)n + 2, 0);
    for (uint32_t o = 0; o < n_op; o++)
        if (def[o] >= 0 && last[o] > def[o]) {
            const int64_t w = opnd_dim(cp.opnd[o]);
            delta[(size_t)def[o] + 1] += w;
            delta[(size_t)last[o] + 1] -= w;
        }
    std::vector<int64_t> live(n + 1, 0);
    {
        int64_t l = 0;
        for (uint32_t j = 0; j <= n; j++) live[j] = (l += delta[j]);
    }
    std::vector<uint64_t> cost(n + 1, 0);  // prefix VALU estimate
    for (uint32_t k = 0; k < n; k++) cost[k + 1] = cost[k] + zxp_instr_cost(cp, k);
    // cuts: near equal work, at the fewest live words within a window
    std::vector<uint32_t> cut = {0};
    const uint64_t total = cost[n];
    for (uint32_t q = 1; q < n_seg; q++) {
        const uint64_t tgt = total * q / n_seg, win = total / (6 * n_seg);
        uint32_t best = 0;
        int64_t bl = INT64_MAX;
        uint64_t bd = UINT64_MAX;
        for (uint32_t j = cut.back() + 1; j < n; j++) {
            if (cost[j] + win < tgt) continue;
            if (cost[j] > tgt + win) break;
            const uint64_t d = cost[j] > tgt ? cost[j] - tgt : tgt - cost[j];
            if (live[j] < bl || (live[j] == bl && d < bd)) {
                bl = live[j];
                bd = d;
                best = j;
            }
        }
        if (best > cut.back()) cut.push_back(best);
    }
    cut.push_back(n);
    const uint32_t S = (uint32_t)cut.size() - 1;
    std::vector<uint32_t> seg_of(n);
    for (uint32_t s = 0; s < S; s++)
        for (uint32_t k = cut[s]; k < cut[s + 1]; k++) seg_of[k] = s;
    // scratch columns of the carried values: busy from the defining segment
    // through the last reading one (a column is reused only by a value
    // defined in a later segment)
    std::vector<int64_t> col_of(n_op, -1);
    {
        std::vector<uint32_t> carried;
        for (uint32_t o = 0; o < n_op; o++)
            if (def[o] >= 0 && last[o] >= 0 && seg_of[last[o]] > seg_of[def[o]]) carried.push_back(o);
        std::stable_sort(carried.begin(), carried.end(), [&](uint32_t x, uint32_t y) { return def[x] < def[y]; });
        std::vector<int64_t> busy;  // per column: last segment that reads it
        for (uint32_t o : carried) {
            const uint32_t w = opnd_dim(cp.opnd[o]), s0 = seg_of[def[o]], s1 = seg_of[last[o]];
            uint32_t c = 0;
            for (;; c++) {
                if (c + w > busy.size()) busy.resize(c + w, -1);
                bool ok = true;
                for (uint32_t j = 0; j < w; j++) ok &= busy[c + j] < (int64_t)s0;
                if (ok) break;
            }
            for (uint32_t j = 0; j < w; j++) busy[c + j] = s1;
            col_of[o] = c;
        }
        n_scratch = (uint32_t)busy.size();
    }
    // emit
    out.resize(S);
    for (uint32_t s = 0; s < S; s++) {
        ZxpSegment &G = out[s];
        G.opnd.assign(cp.opnd, cp.opnd + n_op);
        G.n_tmp1 = cp.n_tmp1;
        G.n_tmp3 = cp.n_tmp3;
        std::vector<uint32_t> scr_op(n_op, UINT32_MAX);   // carried value -> scratch operand
        std::vector<uint32_t> scr_col1(0);                // scratch column -> base COL operand
        auto col1 = [&](uint32_t c) {
            if (c >= scr_col1.size()) scr_col1.resize(c + 1, UINT32_MAX);
            if (scr_col1[c] == UINT32_MAX) {
                scr_col1[c] = (uint32_t)G.opnd.size();
                G.opnd.push_back(zxp_operand{ZXP_COL, ZXP_SEC_SCRATCH, c, 0});
            }
            return scr_col1[c];
        };
        auto scratch = [&](uint32_t o) {
            if (scr_op[o] == UINT32_MAX) {
                if (cp.opnd[o].kind == ZXP_TMP1) {
                    scr_op[o] = col1((uint32_t)col_of[o]);
                } else {
                    scr_op[o] = (uint32_t)G.opnd.size();
                    G.opnd.push_back(zxp_operand{ZXP_COL3, ZXP_SEC_SCRATCH, (uint32_t)col_of[o], 0});
                }
            }
            return scr_op[o];
        };
        std::vector<uint8_t> seen(n_op, 0);
        auto carried_in = [&](uint32_t o) {
            const bool c = is_tmp(cp.opnd[o]) && col_of[o] >= 0 && seg_of[def[o]] < s;
            if (c && !seen[o]) {
                seen[o] = 1;
                G.carry_in += opnd_dim(cp.opnd[o]);
            }
            return c;
        };
        for (uint32_t k = cut[s]; k < cut[s + 1]; k++) {
            zxp_instr I = cp.instr[k];
            if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
                const uint32_t t0 = (uint32_t)G.term.size();
                for (uint32_t t = I.a; t < I.a + I.b; t++) {
                    zxp_term tm = cp.term[t];
                    if (tm.src != ZXP_TERM_ONE && carried_in(tm.src)) {
                        const uint32_t c = (uint32_t)col_of[tm.src] + (cp.opnd[tm.src].kind == ZXP_TMP3 ? tm.comp : 0);
                        tm.src = col1(c);
                        tm.comp = 0;
                    }
                    G.term.push_back(tm);
                }
                I.a = t0;
            } else {
                if (carried_in(I.a)) I.a = scratch(I.a);
                if (I.op != ZXP_COPY && carried_in(I.b)) I.b = scratch(I.b);
            }
            G.instr.push_back(I);
            if (is_tmp(cp.opnd[I.dst]) && col_of[I.dst] >= 0) {  // carried out: stored at its definition
                G.instr.push_back(zxp_instr{ZXP_COPY, scratch(I.dst), I.dst, 0});
                G.carry_out += opnd_dim(cp.opnd[I.dst]);
            }
        }
    }
    return 0;
}

}  // namespace zk
