// Host compiler for ZXP expression programs (include/zkgpu_zxp.h, "compiled
// programs"; C-ABI zkgpu_zxp_compile in include/zkgpu.h).
//
// The reference evaluates its Steps bytecode op by op (step42ns.parser.cpp,
// step52ns.parser.cpp: one AVX2 case per op).  Most of those ops are linear:
// the FRI polynomial (step52ns) is a Horner chain over every committed column
// with challenge v1 plus two Horner chains over the evaluations with v2, and
// the constraint quotient (step42ns) combines every constraint by Horner with
// challenge alpha.  Interpreted literally, each Horner step is a full F_p^3
// product per row.  Here every value is tracked symbolically as an affine form
//     cst + sum_t coef_t * src_t
// over base-field row values src_t (a column at a row shift, or a component
// of an SSA temporary) with row-constant coefficients in F_p^3.  ADD, SUB,
// COPY and MUL-by-a-row-constant fold into the form on the host (exact field
// arithmetic); a form becomes ONE ZXP_DOT instruction only when a row-varying
// product, a column store or the term cap needs its value.  On the device a
// DOT term costs 6 carry-free 32x32 multiply-adds per coefficient component
// (limb form, csrc/gl_device.hpp Dot3) instead of a reduced F_p^3 product.
//
// Hazards: forms refer to SSA temporaries (never overwritten) and to columns;
// before an instruction stores a column, every pending form that reads that
// column is materialised, so reads keep the source program's order.  A stored
// value is first materialised in an SSA temporary; later reads of the same
// (section, column, row shift) in the row use that temporary (store-to-load
// forwarding), so no backend re-reads a cell its own row wrote -- including
// the shifted stores of the reference's stage-3 parsers (step3prev / step3:
// pols[off + ((i+1) % N) * stride] written, then read back, in one row).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/zkgpu.h"

namespace zk {
int set_error(int code, const char *fmt, ...);  // api.hip
}

namespace {

constexpr uint64_t P = 0xFFFFFFFF00000001ULL;
constexpr uint64_t EPS = 0xFFFFFFFFULL;

inline uint64_t canon(uint64_t a) { return a >= P ? a - P : a; }
inline uint64_t fadd(uint64_t a, uint64_t b)
{
    uint64_t s = a + b;  // a, b < P
    return (s < a || s >= P) ? s - P : s;
}
inline uint64_t fsub(uint64_t a, uint64_t b) { return a >= b ? a - b : a + (P - b); }
inline uint64_t fmul(uint64_t a, uint64_t b)
{
    const unsigned __int128 x = (unsigned __int128)a * b;
    const uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
    const uint64_t hh = hi >> 32, hl = hi & EPS;
    uint64_t t0 = lo - hh;
    if (lo < hh) t0 -= EPS;  // borrow: 2^64 == EPS
    const uint64_t t1 = (hl << 32) - hl;
    uint64_t r = t0 + t1;
    if (r < t1) r += EPS;
    return canon(r);
}

struct F3 {
    uint64_t v[3];
    bool zero() const { return !v[0] && !v[1] && !v[2]; }
    bool base() const { return !v[1] && !v[2]; }
};
inline F3 f3(uint64_t a, uint64_t b = 0, uint64_t c = 0) { return F3{{a, b, c}}; }
inline F3 add3(const F3 &a, const F3 &b) { return f3(fadd(a.v[0], b.v[0]), fadd(a.v[1], b.v[1]), fadd(a.v[2], b.v[2])); }
inline F3 sub3(const F3 &a, const F3 &b) { return f3(fsub(a.v[0], b.v[0]), fsub(a.v[1], b.v[1]), fsub(a.v[2], b.v[2])); }
// F_p[x]/(x^3 - x - 1), polinomial.hpp:195-205.  A multiplier with its
// pairwise sums precomputed: the product in 6 base multiplications
// (Karatsuba: c1 = (a0+a1)(b0+b1) - a0b0 - a1b1, ...) instead of 9 -- a
// compiled program scales ~10^5 coefficients by the same constant (scale)
struct Mul3 {
    uint64_t b0, b1, b2, b01, b02, b12;
    bool base;
    explicit Mul3(const F3 &b)
        : b0(b.v[0]), b1(b.v[1]), b2(b.v[2]), b01(fadd(b.v[0], b.v[1])), b02(fadd(b.v[0], b.v[2])),
          b12(fadd(b.v[1], b.v[2])), base(b.base())
    {
    }
    F3 operator()(const F3 &a) const
    {
        if (base) return f3(fmul(a.v[0], b0), fmul(a.v[1], b0), fmul(a.v[2], b0));
        if (a.base()) return f3(fmul(b0, a.v[0]), fmul(b1, a.v[0]), fmul(b2, a.v[0]));
        const uint64_t p0 = fmul(a.v[0], b0), p1 = fmul(a.v[1], b1), p2 = fmul(a.v[2], b2);
        const uint64_t c1 = fsub(fsub(fmul(fadd(a.v[0], a.v[1]), b01), p0), p1);
        const uint64_t c2 = fadd(fsub(fsub(fmul(fadd(a.v[0], a.v[2]), b02), p0), p2), p1);
        const uint64_t c3 = fsub(fsub(fmul(fadd(a.v[1], a.v[2]), b12), p1), p2);
        // x^4 = x^2 + x, x^3 = x + 1
        return f3(fadd(p0, c3), fadd(fadd(c1, p2), c3), fadd(c2, p2));
    }
};

enum { FK_CONST = 0, FK_LIN = 1, FK_SPECIAL = 2 };

struct OKey {
    uint32_t v[4];
    bool operator==(const OKey &o) const { return !memcmp(v, o.v, sizeof(v)); }
};
struct OKeyHash {
    size_t operator()(const OKey &k) const
    {
        uint64_t h = 0x9E3779B97F4A7C15ULL;
        for (uint32_t x : k.v) h = (h ^ x) * 0xBF58476D1CE4E5B9ULL;
        return (size_t)(h ^ (h >> 31));
    }
};

// DOT terms per instruction (Dot3 accumulators stay < 2^63)
constexpr size_t DOT_HARD_CAP = 250;
// A pending form keeps the temporaries it reads alive (LDS slots bound the
// expression kernel's occupancy): flush once it reads more than this many.
constexpr uint32_t MAX_TEMP_REFS = 8;

struct Term {
    uint32_t key;  // output operand index * 4 + component
    F3 c;
};

struct Form {
    uint8_t kind = FK_CONST;
    uint8_t dim = 1;
    int32_t alias = -1;  // output operand holding exactly this value, or -1
    F3 cst = f3(0);
    std::vector<Term> t;  // sorted by key, no zero coefficients
    uint64_t cols = 0;    // Bloom bits (col_bit) of the columns its terms read: a superset
};
inline uint64_t col_bit(uint32_t sec, uint32_t col) { return 1ULL << ((col * 0x9E37u + sec * 31u) & 63u); }

struct Compiler {
    const zxp_instr *in;
    uint32_t n_in;
    const zxp_operand *op;
    const uint64_t *chal, *pub, *evals;
    uint32_t max_terms;
    uint32_t n_src_tmp1, n_src_tmp3;

    std::vector<zxp_operand> opnd;
    std::unordered_map<OKey, uint32_t, OKeyHash> opnd_idx;  // non-temp operands, deduplicated
    std::vector<zxp_instr> instr;
    std::vector<zxp_term> term;
    std::vector<uint64_t> cst;
    std::vector<uint8_t> ssa_kind;  // per output operand: 0 not temp, 1 TMP1 ssa, 3 TMP3 ssa
    uint32_t n_ssa1 = 0, n_ssa3 = 0;
    std::vector<Form> st1, st3;  // current value of every source temporary
    std::vector<uint8_t> set1, set3;
    // output operand of a source COL operand (k) / of COL3 component j (3k + j):
    // intern's answer, kept (a program reads its columns ~10^4 times)
    std::vector<uint32_t> col_out;
    uint32_t col_operand(uint32_t k, uint32_t j)
    {
        const zxp_operand &o = op[k];
        if (col_out.empty()) col_out.assign(3ULL * n_src_opnd, UINT32_MAX);
        uint32_t &r = col_out[3ULL * k + j];
        if (r == UINT32_MAX) r = intern(ZXP_COL, o.a, o.b + j, o.c);
        return r;
    }
    uint32_t n_src_opnd = 0;
    std::unordered_map<OKey, Form, OKeyHash> fwd;  // {sec, col, shift, 0} -> value this row stored there

    uint32_t intern(uint32_t kind, uint32_t a, uint32_t b = 0, uint32_t c = 0)
    {
        const OKey key{{kind, a, b, c}};
        auto it = opnd_idx.find(key);
        if (it != opnd_idx.end()) return it->second;
        opnd.push_back(zxp_operand{kind, a, b, c});
        ssa_kind.push_back(0);
        return opnd_idx[key] = (uint32_t)opnd.size() - 1;
    }

    uint32_t new_ssa(int dim)
    {
        opnd.push_back(zxp_operand{dim == 3 ? (uint32_t)ZXP_TMP3 : (uint32_t)ZXP_TMP1,
                                   dim == 3 ? n_ssa3++ : n_ssa1++, 0, 0});
        ssa_kind.push_back((uint8_t)dim);
        return (uint32_t)opnd.size() - 1;
    }

    uint32_t imm(const F3 &v, int dim)
    {
        cst.insert(cst.end(), v.v, v.v + 3);
        return intern(ZXP_IMM, (uint32_t)(cst.size() / 3 - 1), (uint32_t)dim);
    }

    static Form identity(uint32_t o, int dim)
    {
        Form f;
        f.kind = FK_LIN;
        f.dim = (uint8_t)dim;
        f.alias = (int32_t)o;
        for (int j = 0; j < dim; j++) {
            F3 e = f3(0);
            e.v[j] = 1;
            f.t.push_back(Term{o * 4 + (uint32_t)j, e});
        }
        return f;
    }

    static Form constant(const F3 &v, int dim, int32_t alias)
    {
        Form f;
        f.kind = FK_CONST;
        f.dim = (uint8_t)dim;
        f.cst = v;
        f.alias = alias;
        return f;
    }

    // value of source operand k
    Form load(uint32_t k)
    {
        const zxp_operand &o = op[k];
        switch (o.kind) {
        case ZXP_TMP1: return set1[o.a] ? st1[o.a] : constant(f3(0), 1, -1);
        case ZXP_TMP3: return set3[o.a] ? st3[o.a] : constant(f3(0), 3, -1);
        case ZXP_COL: {
            if (!fwd.empty()) {
                auto it = fwd.find(OKey{{o.a, o.b, o.c, 0}});
                if (it != fwd.end()) return it->second;
            }
            Form f = identity(col_operand(k, 0), 1);
            f.cols = col_bit(o.a, o.b);
            return f;
        }
        case ZXP_COL3: {
            bool any = false;
            for (uint32_t j = 0; j < 3 && !fwd.empty(); j++) any |= fwd.count(OKey{{o.a, o.b + j, o.c, 0}}) != 0;
            if (any) {  // sum_j X^j * component j (forwarded or read)
                Form f = constant(f3(0), 3, -1);
                for (uint32_t j = 0; j < 3; j++) {
                    auto it = fwd.find(OKey{{o.a, o.b + j, o.c, 0}});
                    Form c = it != fwd.end() ? it->second : identity(col_operand(k, j), 1);
                    if (it == fwd.end()) c.cols = col_bit(o.a, o.b + j);
                    F3 e = f3(0);
                    e.v[j] = 1;
                    f = combine(f, scale(c, e, 3), false);
                }
                f.dim = 3;
                f.alias = -1;
                return f;
            }
            Form f;
            f.kind = FK_LIN;
            f.dim = 3;
            f.alias = (int32_t)intern(ZXP_COL3, o.a, o.b, o.c);
            for (uint32_t j = 0; j < 3; j++) {
                F3 e = f3(0);
                e.v[j] = 1;
                f.t.push_back(Term{col_operand(k, j) * 4, e});
                f.cols |= col_bit(o.a, o.b + j);
            }
            for (int a = 1; a < 3; a++)  // (three keys: insertion sort)
                for (int b = a; b > 0 && f.t[b].key < f.t[b - 1].key; b--) std::swap(f.t[b], f.t[b - 1]);
            return f;
        }
        case ZXP_LIT: return constant(f3(((uint64_t)o.a | ((uint64_t)o.b << 32)) % P), 1, intern(ZXP_LIT, o.a, o.b));
        case ZXP_PUB: return constant(f3(pub[o.a] % P), 1, intern(ZXP_PUB, o.a));
        case ZXP_CHAL:
            return constant(f3(chal[3 * o.a] % P, chal[3 * o.a + 1] % P, chal[3 * o.a + 2] % P), 3,
                            intern(ZXP_CHAL, o.a));
        case ZXP_EVAL:
            return constant(f3(evals[3 * o.a] % P, evals[3 * o.a + 1] % P, evals[3 * o.a + 2] % P), 3,
                            intern(ZXP_EVAL, o.a));
        default: {  // X, XDIV, XDIVW, ZI: row-varying values that are not columns
            Form f;
            f.kind = FK_SPECIAL;
            f.dim = (o.kind == ZXP_XDIV || o.kind == ZXP_XDIVW) ? 3 : 1;
            f.alias = (int32_t)intern(o.kind, 0);
            return f;
        }
        }
    }

    // source operand k's value without copying a stored temporary's form
    // (scratch holds the value of any other operand)
    const Form &load_ref(uint32_t k, Form &scratch)
    {
        const zxp_operand &o = op[k];
        if (o.kind == ZXP_TMP1 && set1[o.a]) return st1[o.a];
        if (o.kind == ZXP_TMP3 && set3[o.a]) return st3[o.a];
        scratch = load(k);
        return scratch;
    }

    static void project1(Form &f)
    {
        if (f.dim == 1) return;
        f.dim = 1;
        f.alias = -1;
        f.cst.v[1] = f.cst.v[2] = 0;
        size_t w = 0;
        for (auto &t : f.t) {
            t.c.v[1] = t.c.v[2] = 0;
            if (t.c.v[0]) f.t[w++] = t;
        }
        f.t.resize(w);
        if (f.t.empty()) f.kind = FK_CONST;
    }

    static Form combine(const Form &a, const Form &b, bool sub)
    {
        Form r;
        r.dim = std::max(a.dim, b.dim);
        r.cst = sub ? sub3(a.cst, b.cst) : add3(a.cst, b.cst);
        r.cols = a.cols | b.cols;
        r.t.reserve(a.t.size() + b.t.size());
        size_t i = 0, j = 0;
        while (i < a.t.size() || j < b.t.size()) {
            if (j == b.t.size() || (i < a.t.size() && a.t[i].key < b.t[j].key)) {
                r.t.push_back(a.t[i++]);
            } else if (i == a.t.size() || b.t[j].key < a.t[i].key) {
                const Term &t = b.t[j++];
                r.t.push_back(Term{t.key, sub ? sub3(f3(0), t.c) : t.c});
            } else {
                const F3 c = sub ? sub3(a.t[i].c, b.t[j].c) : add3(a.t[i].c, b.t[j].c);
                if (!c.zero()) r.t.push_back(Term{a.t[i].key, c});
                i++;
                j++;
            }
        }
        r.kind = r.t.empty() ? FK_CONST : FK_LIN;
        return r;
    }

    static Form scale(const Form &a, const F3 &s, int dim)
    {
        Form r;
        r.dim = (uint8_t)dim;
        const Mul3 ms(s);
        r.cst = ms(a.cst);
        r.cols = a.cols;
        if (!s.zero()) {
            r.t.reserve(a.t.size());
            for (const Term &t : a.t) r.t.push_back(Term{t.key, ms(t.c)});
        }
        r.kind = r.t.empty() ? FK_CONST : FK_LIN;
        return r;
    }

    // 1 if every coefficient lies in F_p (the value is a base element)
    static int eff_dim(const Form &f)
    {
        if (!f.cst.base()) return 3;
        for (const Term &t : f.t)
            if (!t.c.base()) return 3;
        return 1;
    }

    void emit_dot(uint32_t dst, Form f)
    {
        // split oversized forms: the first DOT_HARD_CAP terms into a temporary
        while (f.t.size() + 1 > DOT_HARD_CAP) {
            Form part;
            part.kind = FK_LIN;
            part.t.assign(f.t.begin(), f.t.begin() + (DOT_HARD_CAP - 1));
            part.dim = (uint8_t)eff_dim(part);
            const uint32_t t = new_ssa(part.dim);
            emit_dot(t, part);
            Form rest;
            rest.kind = FK_LIN;
            rest.dim = f.dim;
            rest.cst = f.cst;
            rest.t.assign(f.t.begin() + (DOT_HARD_CAP - 1), f.t.end());
            f = combine(rest, identity(t, part.dim), false);
        }
        const uint32_t first = (uint32_t)term.size();
        for (const Term &t : f.t) {
            zxp_term z;
            z.src = t.key >> 2;
            z.comp = t.key & 3;
            memcpy(z.coef, t.c.v, 24);
            term.push_back(z);
        }
        if (!f.cst.zero()) {
            zxp_term z;
            z.src = ZXP_TERM_ONE;
            z.comp = 0;
            memcpy(z.coef, f.cst.v, 24);
            term.push_back(z);
        }
        instr.push_back(zxp_instr{eff_dim(f) == 3 ? (uint32_t)ZXP_DOT3 : (uint32_t)ZXP_DOT1, dst, first,
                                  (uint32_t)term.size() - first});
    }

    // an operand index holding the value of f (emits a DOT into a fresh SSA
    // temporary if needed; f becomes that temporary's identity form)
    uint32_t realize(Form &f)
    {
        if (f.alias >= 0) return (uint32_t)f.alias;
        if (f.kind == FK_CONST) {
            f.alias = (int32_t)imm(f.cst, f.cst.base() ? 1 : 3);
            return (uint32_t)f.alias;
        }
        const int dim = eff_dim(f);
        const uint32_t t = new_ssa(dim);
        emit_dot(t, f);
        f = identity(t, dim);
        return t;
    }

    // distinct SSA temporaries a pending form keeps alive
    uint32_t temp_refs(const Form &f) const
    {
        uint32_t n = 0, last = UINT32_MAX;
        for (const Term &t : f.t) {
            const uint32_t o = t.key >> 2;
            if (ssa_kind[o] && o != last) n++;
            last = o;
        }
        return n;
    }

    bool reads_cols(const Form &f, uint32_t sec, uint32_t c0, uint32_t c1) const
    {
        if (f.kind != FK_LIN) return false;
        for (const Term &t : f.t) {
            const zxp_operand &o = opnd[t.key >> 2];
            if (o.kind == ZXP_COL && o.a == sec && o.b >= c0 && o.b < c1) return true;
        }
        return false;
    }

    // before storing columns [c0, c1) of sec: materialise the pending forms reading them
    void column_hazard(uint32_t sec, uint32_t c0, uint32_t c1)
    {
        uint64_t mask = 0;  // (a form whose Bloom bits miss the stored columns reads none of them)
        for (uint32_t c = c0; c < c1; c++) mask |= col_bit(sec, c);
        for (size_t k = 0; k < st1.size(); k++)
            if (set1[k] && (st1[k].cols & mask) && reads_cols(st1[k], sec, c0, c1)) {
                st1[k].alias = -1;
                realize(st1[k]);
            }
        for (size_t k = 0; k < st3.size(); k++)
            if (set3[k] && (st3[k].cols & mask) && reads_cols(st3[k], sec, c0, c1)) {
                st3[k].alias = -1;
                realize(st3[k]);
            }
    }

    int run()
    {
        st1.assign(n_src_tmp1, Form());
        st3.assign(n_src_tmp3, Form());
        set1.assign(n_src_tmp1, 0);
        set3.assign(n_src_tmp3, 0);
        for (uint32_t k = 0; k < n_in; k++) {
            const zxp_instr &I = in[k];
            const zxp_operand &D = op[I.dst];
            Form sa, sb;
            const Form &A = load_ref(I.a, sa);
            Form R;
            bool opaque = false;
            const Form &B = I.op != ZXP_COPY ? load_ref(I.b, sb) : sb;
            if (I.op == ZXP_COPY) {
                R = A;
            } else if (I.op == ZXP_ADD || I.op == ZXP_SUB) {
                if (A.kind == FK_SPECIAL || B.kind == FK_SPECIAL)
                    opaque = true;
                else
                    R = combine(A, B, I.op == ZXP_SUB);
            } else {  // MUL
                const int dim = std::max(A.dim, B.dim);
                if (A.kind == FK_CONST && B.kind != FK_SPECIAL)
                    R = scale(B, A.cst, dim);
                else if (B.kind == FK_CONST && A.kind != FK_SPECIAL)
                    R = scale(A, B.cst, dim);
                else
                    opaque = true;
            }
            const bool to_col = D.kind == ZXP_COL || D.kind == ZXP_COL3;
            if (opaque) {
                // realise the operands in place (temps keep the realised form)
                const uint32_t ra = realize_src(I.a, sa), rb = realize_src(I.b, sb);
                const int dim = std::max(A.dim, B.dim);
                if (to_col) {
                    const int sd = (D.kind == ZXP_COL || dim == 1) ? 1 : 3;
                    const uint32_t t = opaque_op(I.op, ra, rb, dim);
                    store_col(D, t, sd);
                } else {
                    const int sd = (D.kind == ZXP_TMP1 || dim == 1) ? 1 : 3;
                    store_temp(D, identity(opaque_op(I.op, ra, rb, sd), sd));
                }
                continue;
            }
            if (to_col) {
                if (D.kind == ZXP_COL) project1(R);
                if (R.kind == FK_CONST) {
                    column_hazard(D.a, D.b, D.b + (D.kind == ZXP_COL3 ? 3 : 1));
                    instr.push_back(zxp_instr{ZXP_COPY, intern(D.kind, D.a, D.b, D.c), realize(R), 0});
                    for (uint32_t j = 0; j < (D.kind == ZXP_COL3 ? 3u : 1u); j++)
                        fwd[OKey{{D.a, D.b + j, D.c, 0}}] = constant(f3(R.dim == 3 || j == 0 ? R.cst.v[j] : 0), 1, -1);
                    continue;
                }
                const int rd = eff_dim(R);
                uint32_t t;
                if (R.alias >= 0 && ssa_kind[R.alias] == (uint8_t)rd) {
                    t = (uint32_t)R.alias;
                } else {
                    t = new_ssa(rd);
                    if (R.alias >= 0)
                        instr.push_back(zxp_instr{ZXP_COPY, t, (uint32_t)R.alias, 0});
                    else
                        emit_dot(t, R);
                }
                store_col(D, t, rd);
                continue;
            }
            if (D.kind == ZXP_TMP1) project1(R);
            if (R.kind == FK_LIN && (R.t.size() > max_terms || temp_refs(R) > MAX_TEMP_REFS)) realize(R);
            store_temp(D, std::move(R));
        }
        return 0;
    }

    // A row-varying product (or sum with a special value) of two realised
    // operands into an SSA temporary of dimension dim -- or the temporary that
    // already holds the same operation on the same operands (value numbering:
    // operands are SSA temporaries, or columns / specials read before any
    // store to them -- a column read after a store in the row is the stored
    // SSA value, store_col's forwarding -- so equal operand indices are equal
    // values).  The reference's step3 / step42ns bytecode recompute ~1,300
    // such products each (tools/real_programs_compile.py), which the kernel
    // compiler cannot merge across the kernels' opaque code blocks.
    std::unordered_map<OKey, uint32_t, OKeyHash> vn;
    uint32_t opaque_op(uint32_t opc, uint32_t ra, uint32_t rb, int dim)
    {
        if ((opc == ZXP_MUL || opc == ZXP_ADD) && rb < ra) std::swap(ra, rb);  // commutative
        const OKey key{{opc, ra, rb, (uint32_t)dim}};
        auto it = vn.find(key);
        if (it != vn.end()) return it->second;
        const uint32_t t = new_ssa(dim);
        instr.push_back(zxp_instr{opc, t, ra, rb});
        vn.emplace(key, t);
        return t;
    }

    // realise operand k's value; for temps, the state entry is updated (in
    // place: a reference from load_ref sees the realised form) so later reads
    // reuse the materialised value; any other operand's value is in scratch
    uint32_t realize_src(uint32_t k, Form &scratch)
    {
        const zxp_operand &o = op[k];
        if (o.kind == ZXP_TMP1 && set1[o.a]) return realize(st1[o.a]);
        if (o.kind == ZXP_TMP3 && set3[o.a]) return realize(st3[o.a]);
        return realize(scratch);
    }

    // store SSA temporary t (dimension td) into column operand D (row shift
    // D.c) and remember its components for forwarding
    void store_col(const zxp_operand &D, uint32_t t, int td)
    {
        const uint32_t w = D.kind == ZXP_COL3 ? 3 : 1;
        column_hazard(D.a, D.b, D.b + w);
        instr.push_back(zxp_instr{ZXP_COPY, intern(D.kind, D.a, D.b, D.c), t, 0});
        for (uint32_t j = 0; j < w; j++) {
            Form c;
            if ((int)j < td) {
                c.kind = FK_LIN;
                c.dim = 1;
                c.alias = td == 1 ? (int32_t)t : -1;
                c.t.push_back(Term{t * 4 + j, f3(1)});
            } else {
                c = constant(f3(0), 1, -1);
            }
            fwd[OKey{{D.a, D.b + j, D.c, 0}}] = c;
        }
    }

    void store_temp(const zxp_operand &D, Form f)
    {
        auto &st = D.kind == ZXP_TMP1 ? st1 : st3;
        auto &set = D.kind == ZXP_TMP1 ? set1 : set3;
        st[D.a] = std::move(f);
        set[D.a] = 1;
    }

    // liveness linear scan over the SSA temporaries (two pools)
    void alloc_slots(uint32_t &n_tmp1, uint32_t &n_tmp3)
    {
        const uint32_t n_op = (uint32_t)opnd.size();
        std::vector<uint32_t> first(n_op, UINT32_MAX), last(n_op, 0);
        auto touch = [&](uint32_t o, uint32_t k) {
            if (o >= n_op || !ssa_kind[o]) return;
            first[o] = std::min(first[o], k);
            last[o] = std::max(last[o], k);
        };
        for (uint32_t k = 0; k < instr.size(); k++) {
            const zxp_instr &I = instr[k];
            touch(I.dst, k);
            if (I.op == ZXP_DOT1 || I.op == ZXP_DOT3) {
                for (uint32_t t = I.a; t < I.a + I.b; t++)
                    if (term[t].src != ZXP_TERM_ONE) touch(term[t].src, k);
            } else {
                touch(I.a, k);
                if (I.op != ZXP_COPY) touch(I.b, k);
            }
        }
        for (int pool = 1; pool <= 3; pool += 2) {
            std::vector<uint32_t> order;
            for (uint32_t o = 0; o < n_op; o++)
                if (ssa_kind[o] == pool && first[o] != UINT32_MAX) order.push_back(o);
            std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return first[x] < first[y]; });
            std::vector<uint32_t> slot_end;
            for (uint32_t o : order) {
                uint32_t s = 0;
                while (s < slot_end.size() && slot_end[s] > first[o]) s++;
                if (s == slot_end.size()) slot_end.push_back(0);
                slot_end[s] = last[o];
                opnd[o].a = s;
            }
            (pool == 1 ? n_tmp1 : n_tmp3) = (uint32_t)std::max<size_t>(slot_end.size(), 1);
        }
    }
};


// ---------------------------------------------------------------- scheduling
// The source order of a large program can keep hundreds of values alive: the
// reference's step42ns bytecode (zkevm.chelpers.step42ns.parser.hpp) first
// computes every constraint value and only then folds them with the alpha
// Horner chain (fused opcodes 84/87), so ~1,190 base + 174 extension
// temporaries are live at once -- far beyond a GPU thread's registers.  The
// program is a DAG: every temporary write is an SSA definition, column
// stores are ordered sinks.  It is re-emitted sink by sink in depth-first
// post-order, visiting the operand that needs the most registers first
// (Sethi-Ullman), so each constraint is evaluated right before its use; on
// the fork-9 step42ns this takes the peak from ~1,670 live words to ~100.
// Memory order is kept: a column store follows every earlier read and store
// of that column, a read follows the last earlier store of its column.
// Values no sink depends on are dropped.
struct Scheduled {
    std::vector<zxp_instr> instr;
    std::vector<zxp_operand> opnd;
    uint32_t n_tmp1 = 0, n_tmp3 = 0;
};

static void schedule(const zxp_instr *in, uint32_t n_in, const zxp_operand *op, uint32_t n_opnd, uint32_t n_tmp1,
                     uint32_t n_tmp3, Scheduled &out)
{
    out.opnd.assign(op, op + n_opnd);
    // never-written temporaries read as zero: one shared zero slot per pool
    const uint32_t zero1 = (uint32_t)out.opnd.size();
    out.opnd.push_back(zxp_operand{ZXP_TMP1, 0, 0, 0});
    const uint32_t zero3 = (uint32_t)out.opnd.size();
    out.opnd.push_back(zxp_operand{ZXP_TMP3, 0, 0, 0});
    uint32_t v1 = 1, v3 = 1;  // SSA versions (slot 0 of each pool = the zero temporary)
    std::vector<int64_t> def1(n_tmp1, -1), def3(n_tmp3, -1);  // slot -> defining instruction
    std::vector<uint32_t> dop(n_in);                          // instruction -> its SSA destination operand
    std::vector<std::vector<uint32_t>> deps(n_in);
    std::vector<zxp_instr> ren(in, in + n_in);
    std::vector<uint8_t> width(n_in, 0), sink(n_in, 0);
    struct ColState {
        int64_t last_store = -1;
        std::vector<uint32_t> reads;
    };
    std::unordered_map<uint64_t, ColState> cols;
    auto colkey = [](uint32_t sec, uint32_t c) { return ((uint64_t)sec << 32) | c; };
    for (uint32_t k = 0; k < n_in; k++) {
        const zxp_instr &I = in[k];
        auto use = [&](uint32_t x) -> uint32_t {
            const zxp_operand &o = op[x];
            if (o.kind == ZXP_TMP1 || o.kind == ZXP_TMP3) {
                const int64_t d = o.kind == ZXP_TMP1 ? def1[o.a] : def3[o.a];
                if (d < 0) return o.kind == ZXP_TMP1 ? zero1 : zero3;
                deps[k].push_back((uint32_t)d);
                return dop[d];
            }
            if (o.kind == ZXP_COL || o.kind == ZXP_COL3)
                for (uint32_t c = 0; c < (o.kind == ZXP_COL3 ? 3u : 1u); c++) {
                    ColState &cs = cols[colkey(o.a, o.b + c)];
                    if (cs.last_store >= 0) deps[k].push_back((uint32_t)cs.last_store);
                    cs.reads.push_back(k);
                }
            return x;
        };
        ren[k].a = use(I.a);
        if (I.op != ZXP_COPY) ren[k].b = use(I.b);
        const zxp_operand &D = op[I.dst];
        if (D.kind == ZXP_TMP1 || D.kind == ZXP_TMP3) {
            const bool t3 = D.kind == ZXP_TMP3;
            dop[k] = (uint32_t)out.opnd.size();
            out.opnd.push_back(zxp_operand{D.kind, t3 ? v3++ : v1++, 0, 0});
            (t3 ? def3[D.a] : def1[D.a]) = k;
            width[k] = t3 ? 3 : 1;
            ren[k].dst = dop[k];
        } else {  // column store: an ordered sink
            sink[k] = 1;
            for (uint32_t c = 0; c < (D.kind == ZXP_COL3 ? 3u : 1u); c++) {
                ColState &cs = cols[colkey(D.a, D.b + c)];
                if (cs.last_store >= 0) deps[k].push_back((uint32_t)cs.last_store);
                for (uint32_t r : cs.reads)
                    if (r != k) deps[k].push_back(r);
                cs.reads.clear();
                cs.last_store = k;
            }
        }
        std::sort(deps[k].begin(), deps[k].end());
        deps[k].erase(std::unique(deps[k].begin(), deps[k].end()), deps[k].end());
    }
    // register need, bottom-up (deps have smaller indices)
    std::vector<uint32_t> need(n_in, 0);
    std::vector<uint32_t> order;
    for (uint32_t k = 0; k < n_in; k++) {
        std::vector<uint32_t> &d = deps[k];
        std::stable_sort(d.begin(), d.end(), [&](uint32_t x, uint32_t y) { return need[x] > need[y]; });
        uint32_t held = 0, nd = width[k];
        for (uint32_t c : d) {
            nd = std::max(nd, held + need[c]);
            held += width[c];
        }
        need[k] = nd;
    }
    // emit: sinks in source order, each after its unscheduled dependencies
    // (iterative depth-first post-order, highest need first)
    std::vector<uint8_t> done(n_in, 0);
    std::vector<std::pair<uint32_t, uint32_t>> stack;
    for (uint32_t s = 0; s < n_in; s++) {
        if (!sink[s] || done[s]) continue;
        stack.push_back({s, 0});
        while (!stack.empty()) {
            auto &top = stack.back();
            const uint32_t k = top.first;
            if (top.second < deps[k].size()) {
                const uint32_t c = deps[k][top.second++];
                if (!done[c]) {
                    done[c] = 2;  // on the stack (a DAG: no cycles)
                    stack.push_back({c, 0});
                }
                continue;
            }
            done[k] = 1;
            order.push_back(k);
            stack.pop_back();
        }
    }
    out.instr.clear();
    out.instr.reserve(order.size());
    for (uint32_t k : order) out.instr.push_back(ren[k]);
    out.n_tmp1 = v1;
    out.n_tmp3 = v3;
}

struct Out {
    std::vector<zxp_instr> instr;
    std::vector<zxp_operand> opnd;
    std::vector<zxp_term> term;
    std::vector<uint64_t> cst;
};
thread_local Out g_out;

// Peak temporary words (1 per base, 3 per extension value) live at once in
// the source order: every definition of a slot lives to its last read
// before the slot's next definition.
uint32_t source_peak_live(const zxp_instr *in, uint32_t n, const zxp_operand *op)
{
    std::vector<int64_t> delta((size_t)n + 2, 0);
    std::map<std::pair<uint32_t, uint32_t>, std::pair<uint32_t, uint32_t>> cur;  // slot -> [def, last read]
    auto width = [](uint32_t kind) { return kind == ZXP_TMP3 ? 3 : 1; };
    auto close = [&](const std::pair<uint32_t, uint32_t> &key, const std::pair<uint32_t, uint32_t> &iv) {
        delta[iv.first] += width(key.first);
        delta[(size_t)iv.second + 1] -= width(key.first);
    };
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t srcs[2] = {in[k].a, in[k].b};
        for (int j = 0; j < (in[k].op == ZXP_COPY ? 1 : 2); j++) {
            const zxp_operand &o = op[srcs[j]];
            if (o.kind != ZXP_TMP1 && o.kind != ZXP_TMP3) continue;
            auto it = cur.find({o.kind, o.a});
            if (it != cur.end()) it->second.second = k;
        }
        const zxp_operand &d = op[in[k].dst];
        if (d.kind == ZXP_TMP1 || d.kind == ZXP_TMP3) {
            const std::pair<uint32_t, uint32_t> key{d.kind, d.a};
            auto it = cur.find(key);
            if (it != cur.end()) close(key, it->second);
            cur[key] = {k, k};
        }
    }
    for (const auto &kv : cur) close(kv.first, kv.second);
    int64_t live = 0, peak = 0;
    for (size_t k = 0; k < delta.size(); k++) peak = std::max(peak, live += delta[k]);
    return (uint32_t)peak;
}

// The register-pressure decision and the schedule depend only on the source
// program's structure (instructions, operand table, temporary pools), never on
// the challenge / public / eval values -- and a prover compiles the same stage
// programs every proof (18 ms of the zkEVM-shaped quotient's ~40 ms host
// compile).  They are kept per process, keyed by the program's bytes (compared
// in full on a hit), at most SCHED_MEMO entries.
struct SchedMemo {
    std::vector<zxp_instr> in;
    std::vector<zxp_operand> op;
    uint32_t n_tmp1 = 0, n_tmp3 = 0;
    bool sched_on = false;
    Scheduled sp;
};
constexpr size_t SCHED_MEMO = 32;

static uint64_t program_hash(const zxp_instr *in, uint32_t n_in, const zxp_operand *op, uint32_t n_opnd)
{
    uint64_t h = 0x9E3779B97F4A7C15ULL ^ ((uint64_t)n_in << 32 | n_opnd);
    auto mix = [&](const void *p, size_t bytes) {
        const uint8_t *b = (const uint8_t *)p;
        size_t k = 0;
        for (; k + 8 <= bytes; k += 8) {
            uint64_t w;
            memcpy(&w, b + k, 8);
            h = (h ^ w) * 0xBF58476D1CE4E5B9ULL;
            h ^= h >> 31;
        }
        for (; k < bytes; k++) h = (h ^ b[k]) * 0x100000001B3ULL;
    };
    mix(in, (size_t)n_in * sizeof(zxp_instr));
    mix(op, (size_t)n_opnd * sizeof(zxp_operand));
    return h;
}

static std::shared_ptr<const SchedMemo> scheduled_program(const zxp_instr *in, uint32_t n_in, const zxp_operand *op,
                                                          uint32_t n_opnd, uint32_t n_tmp1, uint32_t n_tmp3)
{
    static std::mutex mu;
    static std::unordered_map<uint64_t, std::shared_ptr<const SchedMemo>> memo;
    const uint64_t key = program_hash(in, n_in, op, n_opnd) ^ ((uint64_t)n_tmp1 << 20) ^ ((uint64_t)n_tmp3 << 40);
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = memo.find(key);
        if (it != memo.end()) {
            const SchedMemo &m = *it->second;
            if (m.in.size() == n_in && m.op.size() == n_opnd && m.n_tmp1 == n_tmp1 && m.n_tmp3 == n_tmp3 &&
                !memcmp(m.in.data(), in, (size_t)n_in * sizeof(zxp_instr)) &&
                !memcmp(m.op.data(), op, (size_t)n_opnd * sizeof(zxp_operand)))
                return it->second;
        }
    }
    auto m = std::make_shared<SchedMemo>();
    m->in.assign(in, in + n_in);
    m->op.assign(op, op + n_opnd);
    m->n_tmp1 = n_tmp1;
    m->n_tmp3 = n_tmp3;
    // reschedule for register pressure when the source order keeps more than
    // 96 temporary words live (the zkEVM's bytecode: ~1,200); otherwise keep
    // the producer's order, in which each constraint is folded into the
    // accumulator as soon as it is computed (the 2^23 config-4 quotient: 186
    // VGPRs in source order, 512 + spills scheduled).
    m->sched_on = source_peak_live(in, n_in, op) > 96;
    if (m->sched_on) schedule(in, n_in, op, n_opnd, n_tmp1, n_tmp3, m->sp);
    std::lock_guard<std::mutex> lk(mu);
    if (memo.size() >= SCHED_MEMO) memo.clear();
    memo[key] = m;
    return m;
}

}  // namespace

extern "C" int zkgpu_zxp_compile(const void *instr, uint32_t n_instr, const void *opnd, uint32_t n_opnd,
                                 uint32_t n_tmp1, uint32_t n_tmp3, const uint64_t *challenges,
                                 const uint64_t *publics, uint32_t n_publics, const uint64_t *evals, uint32_t n_evals,
                                 uint32_t max_terms, zxp_compiled *out)
{
    using zk::set_error;
    if (!out || (n_instr && (!instr || !opnd))) return set_error(ZKGPU_ERR_ARG, "zxp_compile: null argument");
    if (max_terms == 0) max_terms = 64;
    if (max_terms > 256) max_terms = 256;  // Dot3 accumulators: < 2^63 for 256 terms + constant
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
        case ZXP_CHAL: bad = o.a >= 8 || !challenges; break;
        case ZXP_PUB: bad = o.a >= n_publics || !publics; break;
        case ZXP_EVAL: bad = o.a >= n_evals || !evals; break;
        case ZXP_COL:
        case ZXP_COL3:
        case ZXP_LIT:
        case ZXP_X:
        case ZXP_XDIV:
        case ZXP_XDIVW:
        case ZXP_ZI: break;
        default: bad = true;
        }
        if (bad) return set_error(ZKGPU_ERR_ARG, "zxp: operand %u (kind %u) invalid", k, o.kind);
    }
    for (uint32_t k = 0; k < n_instr; k++) {
        const uint32_t dk = op[in[k].dst].kind;
        if (dk != ZXP_TMP1 && dk != ZXP_TMP3 && dk != ZXP_COL && dk != ZXP_COL3)
            return set_error(ZKGPU_ERR_ARG, "zxp: instruction %u writes a read-only operand", k);
    }
    // the schedule (structure only, kept per process: scheduled_program)
    const std::shared_ptr<const SchedMemo> memo = scheduled_program(in, n_instr, op, n_opnd, n_tmp1, n_tmp3);
    if (memo->sched_on) {
        const Scheduled &sp = memo->sp;
        in = sp.instr.data();
        n_instr = (uint32_t)sp.instr.size();
        op = sp.opnd.data();
        n_opnd = (uint32_t)sp.opnd.size();
        n_tmp1 = sp.n_tmp1;
        n_tmp3 = sp.n_tmp3;
    }
    Compiler c;
    c.in = in;
    c.n_in = n_instr;
    c.op = op;
    c.chal = challenges;
    c.pub = publics;
    c.evals = evals;
    c.max_terms = max_terms;
    c.n_src_tmp1 = n_tmp1;
    c.n_src_opnd = n_opnd;
    c.n_src_tmp3 = n_tmp3;
    c.run();
    uint32_t t1 = 1, t3 = 1;
    c.alloc_slots(t1, t3);
    g_out.instr.swap(c.instr);
    g_out.opnd.swap(c.opnd);
    g_out.term.swap(c.term);
    g_out.cst.swap(c.cst);
    out->instr = g_out.instr.data();
    out->n_instr = (uint32_t)g_out.instr.size();
    out->opnd = g_out.opnd.data();
    out->n_opnd = (uint32_t)g_out.opnd.size();
    out->term = g_out.term.data();
    out->n_term = (uint32_t)g_out.term.size();
    out->cst = g_out.cst.data();
    out->n_cst = (uint32_t)(g_out.cst.size() / 3);
    out->n_tmp1 = t1;
    out->n_tmp3 = t3;
    return 0;
}
