// StarkInfo JSON loader and its translation into the GPU prover's instance
// description.  See zkgpu_stark_info.hpp.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <tuple>

#include "zkgpu_stark_info.hpp"

namespace zkgpu {

static const uint64_t GL_P = 0xFFFFFFFF00000001ULL;

const char *const SECTION_NAMES[S_MAX] = {"cm1_n",   "cm1_2ns", "cm2_n",    "cm2_2ns", "cm3_n", "cm3_2ns",
                                          "cm4_n",   "cm4_2ns", "tmpExp_n", "q_2ns",   "f_2ns"};

// stark_info.cpp:484-511
ESection string2section(const std::string &s)
{
    for (int k = 0; k < S_MAX; k++)
        if (s == SECTION_NAMES[k]) return (ESection)k;
    throw std::runtime_error("string2section() found invalid string=" + s);
}

static void load_sections(const json::Value &j, uint64_t out[S_MAX])
{
    // the eleven keys stark_info.cpp:46-129 reads per PolsSections
    for (int k = 0; k < S_MAX; k++) out[k] = j[SECTION_NAMES[k]].u64();
}

static StepTypeJ load_type(const json::Value &j, bool is_dest)
{
    static const char *const TYPES[] = {"tmp",    "exp",        "eval",        "challenge", "tree1", "tree2", "tree3",
                                        "tree4",  "number",     "x",           "Z",         "public", "xDivXSubXi",
                                        "xDivXSubWXi", "cm",    "const",       "q",         "Zi",    "tmpExp", "f"};
    StepTypeJ t;
    t.type = j["type"].string();
    bool ok = false;
    for (const char *n : TYPES) ok |= t.type == n;
    if (!ok) throw std::runtime_error("StepType::setType() found invalid type: " + t.type);
    if (is_dest) t.id = j["id"].u64();  // mandatory for the destination
    else t.id = j.contains("id") ? j["id"].u64() : 0;
    t.prime = j.contains("prime") ? j["prime"].boolean() : false;
    t.p = j.contains("p") ? j["p"].u64() : 0;
    if (j.contains("value")) t.value = j["value"].kind == json::Value::String ? j["value"].s : j["value"].s;
    return t;
}

// stark_info.cpp:197-398 (every step: "op", "dest", "src"; "first" code)
static StepJ load_step(const json::Value &j)
{
    StepJ st;
    st.tmpUsed = j["tmpUsed"].u64();
    const json::Value &f = j["first"];
    for (size_t i = 0; i < f.size(); i++) {
        StepOperationJ op;
        op.op = f[i]["op"].string();
        if (op.op != "add" && op.op != "sub" && op.op != "mul" && op.op != "copy")
            throw std::runtime_error("StepOperation::setOperation() found invalid type: " + op.op);
        op.dest = load_type(f[i]["dest"], true);
        const json::Value &src = f[i]["src"];
        for (size_t k = 0; k < src.size(); k++) op.src.push_back(load_type(src[k], false));
        st.first.push_back(std::move(op));
    }
    return st;
}

static std::vector<uint64_t> load_nullable(const json::Value &j)
{
    std::vector<uint64_t> v;
    for (size_t i = 0; i < j.size(); i++) v.push_back(j[i].is_null() ? 0 : j[i].u64());
    return v;
}

void StarkInfo::load(const json::Value &j)
{
    const json::Value &ss = j["starkStruct"];
    nBits = ss["nBits"].u64();
    nBitsExt = ss["nBitsExt"].u64();
    nQueries = ss["nQueries"].u64();
    verificationHashType = ss["verificationHashType"].string();
    for (size_t i = 0; i < ss["steps"].size(); i++) stepsNBits.push_back(ss["steps"][i]["nBits"].u64());

    mapTotalN = j["mapTotalN"].u64();
    nConstants = j["nConstants"].u64();
    nPublics = j["nPublics"].u64();
    nCm1 = j["nCm1"].u64();
    nCm2 = j["nCm2"].u64();
    nCm3 = j["nCm3"].u64();
    nCm4 = j["nCm4"].u64();
    friExpId = j["friExpId"].u64();
    nExps = j["nExps"].u64();
    qDim = j["qDim"].u64();
    qDeg = j["qDeg"].u64();

    load_sections(j["mapDeg"], mapDeg);
    load_sections(j["mapOffsets"], mapOffsets);
    for (int k = 0; k < S_MAX; k++) {
        const json::Value &v = j["mapSections"][SECTION_NAMES[k]];
        for (size_t i = 0; i < v.size(); i++) mapSections[k].push_back(v[i].u64());
    }
    load_sections(j["mapSectionsN"], mapSectionsN);
    load_sections(j["mapSectionsN1"], mapSectionsN1);
    load_sections(j["mapSectionsN3"], mapSectionsN3);

    for (size_t i = 0; i < j["varPolMap"].size(); i++) {
        const json::Value &v = j["varPolMap"][i];
        varPolMap.push_back(VarPolMapJ{string2section(v["section"].string()), v["dim"].u64(), v["sectionPos"].u64()});
    }
    for (size_t i = 0; i < j["qs"].size(); i++) qs.push_back(j["qs"][i].u64());
    for (size_t i = 0; i < j["cm_n"].size(); i++) cm_n.push_back(j["cm_n"][i].u64());
    for (size_t i = 0; i < j["cm_2ns"].size(); i++) cm_2ns.push_back(j["cm_2ns"][i].u64());
    for (size_t i = 0; i < j["peCtx"].size(); i++) {
        const json::Value &v = j["peCtx"][i];
        peCtx.push_back(PeCtxJ{v["tExpId"].u64(), v["fExpId"].u64(), v["zId"].u64(), v["c1Id"].u64(),
                               v["numId"].u64(), v["denId"].u64(), v["c2Id"].u64()});
    }
    for (size_t i = 0; i < j["puCtx"].size(); i++) {
        const json::Value &v = j["puCtx"][i];
        puCtx.push_back(PuCtxJ{v["tExpId"].u64(), v["fExpId"].u64(), v["h1Id"].u64(), v["h2Id"].u64(),
                               v["zId"].u64(), v["c1Id"].u64(), v["numId"].u64(), v["denId"].u64(),
                               v["c2Id"].u64()});
    }
    for (size_t i = 0; i < j["ciCtx"].size(); i++) {
        const json::Value &v = j["ciCtx"][i];
        ciCtx.push_back(CiCtxJ{v["zId"].u64(), v["numId"].u64(), v["denId"].u64(), v["c1Id"].u64(),
                               v["c2Id"].u64()});
    }
    for (size_t i = 0; i < j["evMap"].size(); i++) {
        const json::Value &v = j["evMap"][i];
        const std::string &t = v["type"].string();
        EvMapJ e;
        if (t == "cm") e.type = EvMapJ::cm;
        else if (t == "const") e.type = EvMapJ::_const;
        else if (t == "q") e.type = EvMapJ::q;
        else throw std::runtime_error("EvMap::setType() found invalid type: " + t);
        e.id = v["id"].u64();
        e.prime = v["prime"].boolean();
        evMap.push_back(e);
    }
    step2prev = load_step(j["step2prev"]);
    step3prev = load_step(j["step3prev"]);
    step3 = load_step(j["step3"]);
    step42ns = load_step(j["step42ns"]);
    step52ns = load_step(j["step52ns"]);
    exps_n = load_nullable(j["exps_n"]);
    q_2nsVector = load_nullable(j["q_2ns"]);
    cm4_nVector = load_nullable(j["cm4_n"]);
    cm4_2nsVector = load_nullable(j["cm4_2ns"]);
    tmpExp_n = load_nullable(j["tmpExp_n"]);
    const json::Value &e2p = j["exp2pol"];
    for (const auto &kv : e2p.o) exp2pol[kv.first] = kv.second.u64();
}

StarkInfo StarkInfo::from_file(const std::string &path)
{
    std::ifstream f(path);
    if (!f.good()) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    StarkInfo si;
    si.load(json::parse(ss.str()));
    return si;
}

// ---------------------------------------------------------------- translation
zkgpu_zxp_prog ZxpProgram::view() const
{
    zkgpu_zxp_prog p;
    p.instr = instr.data();
    p.n_instr = (uint32_t)instr.size();
    p.opnd = opnd.data();
    p.n_opnd = (uint32_t)opnd.size();
    p.n_tmp1 = n_tmp1;
    p.n_tmp3 = n_tmp3;
    return p;
}

// the GPU sections (include/zkgpu_zxp.h) of the reference's eSection
static int zxp_section(ESection s)
{
    switch (s) {
    case S_CM1_N: return SEC_CM1_N;
    case S_CM2_N: return SEC_CM2_N;
    case S_CM3_N: return SEC_CM3_N;
    case S_TMPEXP_N: return SEC_TMP_N;
    case S_CM1_2NS: return SEC_CM1_2NS;
    case S_CM2_2NS: return SEC_CM2_2NS;
    case S_CM3_2NS: return SEC_CM3_2NS;
    case S_CM4_2NS: return SEC_CM4_2NS;
    case S_Q_2NS: return SEC_Q_2NS;
    case S_F_2NS: return SEC_F_2NS;
    default: return -1;  // cm4_n: not a section the expression programs address
    }
}

static const VarPolMapJ &pol(const StarkInfo &si, uint64_t id, const char *what)
{
    if (id >= si.varPolMap.size()) throw std::runtime_error(std::string(what) + ": polynomial id out of range");
    return si.varPolMap[id];
}

static uint64_t exp_pol(const StarkInfo &si, uint64_t expId, const char *what)
{
    auto it = si.exp2pol.find(std::to_string(expId));
    if (it == si.exp2pol.end()) throw std::runtime_error(std::string(what) + ": expression " + std::to_string(expId) + " has no polynomial (exp2pol)");
    return it->second;
}

namespace {
struct Conv {
    const StarkInfo &si;
    bool ext;
    const char *name;
    ZxpProgram prog;
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, uint32_t> index;
    std::map<uint64_t, uint32_t> tmp_dim;  // tmp id -> dim of its current value

    [[noreturn]] void bad(const std::string &m) const
    {
        throw std::runtime_error(std::string(name) + ": " + m);
    }
    uint32_t operand(uint32_t kind, uint32_t a = 0, uint32_t b = 0, uint32_t c = 0)
    {
        auto key = std::make_tuple(kind, a, b, c);
        auto it = index.find(key);
        if (it != index.end()) return it->second;
        const uint32_t k = (uint32_t)prog.opnd.size();
        prog.opnd.push_back(zxp_operand{kind, a, b, c});
        index[key] = k;
        return k;
    }
    uint32_t shift(bool prime) const { return prime ? (ext ? 1u << (si.nBitsExt - si.nBits) : 1u) : 0u; }
    // a column operand of polynomial polId
    uint32_t polcol(uint64_t polId, bool prime, uint32_t &dim, const char *what)
    {
        const VarPolMapJ &m = pol(si, polId, what);
        const int sec = zxp_section(m.section);
        if (sec < 0) bad(std::string(what) + ": section " + SECTION_NAMES[m.section] + " is not addressable");
        const bool sec_ext = sec >= SEC_CM1_2NS;
        if (sec_ext != ext) bad(std::string(what) + ": section " + SECTION_NAMES[m.section] + " is on the other domain");
        if (m.dim != 1 && m.dim != 3) bad("polynomial dimension must be 1 or 3");
        dim = (uint32_t)m.dim;
        return operand(dim == 3 ? ZXP_COL3 : ZXP_COL, (uint32_t)sec, (uint32_t)m.sectionPos, shift(prime));
    }
    uint32_t src(const StepTypeJ &t, uint32_t &dim)
    {
        const std::string &ty = t.type;
        if (ty == "tmp") {
            auto it = tmp_dim.find(t.id);
            if (it == tmp_dim.end()) bad("tmp " + std::to_string(t.id) + " read before written");
            dim = it->second;
            return operand(dim == 3 ? ZXP_TMP3 : ZXP_TMP1, (uint32_t)t.id);
        }
        if (ty == "cm") {
            const std::vector<uint64_t> &cm = ext ? si.cm_2ns : si.cm_n;
            if (t.id >= cm.size()) bad("cm id out of range");
            return polcol(cm[t.id], t.prime, dim, "cm");
        }
        if (ty == "exp") {
            if (ext) bad("exp operands are n-domain expressions (tmpExp_n)");
            return polcol(exp_pol(si, t.id, name), t.prime, dim, "exp");
        }
        if (ty == "const") {
            if (t.id >= si.nConstants) bad("const id out of range");
            dim = 1;
            return operand(ZXP_COL, ext ? SEC_CONST_2NS : SEC_CONST_N, (uint32_t)t.id, shift(t.prime));
        }
        if (ty == "number") {
            // pil-stark writes literals as decimal strings (negative values mod p)
            const std::string &s = t.value;
            if (s.empty()) bad("number without value");
            const bool neg = s[0] == '-';
            unsigned __int128 v = 0;
            for (size_t i = neg ? 1 : 0; i < s.size(); i++) {
                if (s[i] < '0' || s[i] > '9') bad("bad number " + s);
                v = (v * 10 + (unsigned)(s[i] - '0')) % GL_P;
            }
            uint64_t x = (uint64_t)v;
            if (neg && x) x = GL_P - x;
            dim = 1;
            return operand(ZXP_LIT, (uint32_t)x, (uint32_t)(x >> 32));
        }
        if (ty == "public") {
            if (t.id >= si.nPublics) bad("public id out of range");
            dim = 1;
            return operand(ZXP_PUB, (uint32_t)t.id);
        }
        if (ty == "challenge") {
            if (t.id >= 8) bad("challenge id out of range");
            dim = 3;
            return operand(ZXP_CHAL, (uint32_t)t.id);
        }
        if (ty == "eval") {
            if (t.id >= si.evMap.size()) bad("eval id out of range");
            dim = 3;
            return operand(ZXP_EVAL, (uint32_t)t.id);
        }
        if (ty == "x") {
            dim = 1;
            return operand(ZXP_X);
        }
        if (ty == "Zi") {
            if (!ext) bad("Zi is a 2ns-domain operand");
            dim = 1;
            return operand(ZXP_ZI);
        }
        if (ty == "xDivXSubXi" || ty == "xDivXSubWXi") {
            if (!ext) bad(ty + " is a 2ns-domain operand");
            dim = 3;
            return operand(ty == "xDivXSubXi" ? ZXP_XDIV : ZXP_XDIVW);
        }
        bad("operand type " + ty + " is not taken by the GPU programs");
    }
    uint32_t dest(const StepTypeJ &t, uint32_t rdim)
    {
        const std::string &ty = t.type;
        if (ty == "tmp") {
            tmp_dim[t.id] = rdim;
            if (rdim == 3) prog.n_tmp3 = std::max<uint32_t>(prog.n_tmp3, (uint32_t)t.id + 1);
            else prog.n_tmp1 = std::max<uint32_t>(prog.n_tmp1, (uint32_t)t.id + 1);
            return operand(rdim == 3 ? ZXP_TMP3 : ZXP_TMP1, (uint32_t)t.id);
        }
        uint32_t d = 0, k;
        if (ty == "cm") {
            const std::vector<uint64_t> &cm = ext ? si.cm_2ns : si.cm_n;
            if (t.id >= cm.size()) bad("cm id out of range");
            k = polcol(cm[t.id], t.prime, d, "cm");
        } else if (ty == "exp") {
            if (ext) bad("exp destinations are n-domain expressions (tmpExp_n)");
            k = polcol(exp_pol(si, t.id, name), t.prime, d, "exp");
        } else if (ty == "q" || ty == "f") {
            if (!ext) bad(ty + " is a 2ns-domain destination");
            d = (uint32_t)si.qDim;
            if (d != 1 && d != 3) bad("qDim must be 1 or 3");
            k = operand(d == 3 ? ZXP_COL3 : ZXP_COL, ty == "q" ? SEC_Q_2NS : SEC_F_2NS, 0, shift(t.prime));
        } else {
            bad("destination type " + ty + " is not taken by the GPU programs");
        }
        if (rdim > d) bad("an F_p^3 value stored to a base-field column");
        return k;
    }
};
}  // namespace

ZxpProgram step_to_zxp(const StarkInfo &si, const StepJ &step, bool ext, const char *name)
{
    Conv c{si, ext, name, {}, {}, {}};
    for (const StepOperationJ &o : step.first) {
        const uint32_t op = o.op == "add" ? ZXP_ADD : o.op == "sub" ? ZXP_SUB : o.op == "mul" ? ZXP_MUL : ZXP_COPY;
        const size_t want = op == ZXP_COPY ? 1 : 2;
        if (o.src.size() != want) c.bad("operation " + o.op + " takes " + std::to_string(want) + " sources");
        uint32_t da = 0, db = 0;
        const uint32_t a = c.src(o.src[0], da);
        const uint32_t b = want == 2 ? c.src(o.src[1], db) : 0;
        const uint32_t rdim = std::max(da, db);
        const uint32_t d = c.dest(o.dest, rdim);
        c.prog.instr.push_back(zxp_instr{op, d, a, b});
    }
    return std::move(c.prog);
}

ProverInfo::ProverInfo(const StarkInfo &si)
{
    memset(&info_, 0, sizeof info_);
    if (si.qDim != 3) throw std::runtime_error("StarkInfo: qDim must be 3 (F_p^3 quotient)");
    if (si.stepsNBits.empty() || si.stepsNBits.size() > 32) throw std::runtime_error("StarkInfo: 1..32 FRI steps");
    info_.n_bits = (uint32_t)si.nBits;
    info_.n_bits_ext = (uint32_t)si.nBitsExt;
    info_.n_queries = (uint32_t)si.nQueries;
    info_.n_fri_steps = (uint32_t)si.stepsNBits.size();
    for (size_t i = 0; i < si.stepsNBits.size(); i++) info_.fri_steps[i] = (uint32_t)si.stepsNBits[i];
    info_.n_cm1 = (uint32_t)si.mapSectionsN[S_CM1_N];
    info_.n_cm2 = (uint32_t)si.mapSectionsN[S_CM2_N];
    info_.n_cm3 = (uint32_t)si.mapSectionsN[S_CM3_N];
    info_.n_cm4 = (uint32_t)si.mapSectionsN[S_CM4_2NS];
    info_.n_tmp = (uint32_t)si.mapSectionsN[S_TMPEXP_N];
    info_.n_const = (uint32_t)si.nConstants;
    info_.n_publics = (uint32_t)si.nPublics;
    info_.q_deg = (uint32_t)si.qDeg;
    // evMap (starks.cpp:563-582): cm -> cm_2ns[id], const -> column id, q -> qs[id]
    for (size_t i = 0; i < si.evMap.size(); i++) {
        const EvMapJ &e = si.evMap[i];
        uint32_t sec, col, dim;
        if (e.type == EvMapJ::_const) {
            sec = SEC_CONST_2NS;
            col = (uint32_t)e.id;
            dim = 1;
        } else {
            const std::vector<uint64_t> &ids = e.type == EvMapJ::cm ? si.cm_2ns : si.qs;
            if (e.id >= ids.size()) throw std::runtime_error("evMap: id out of range");
            const VarPolMapJ &m = pol(si, ids[e.id], "evMap");
            const int s = zxp_section(m.section);
            if (s < SEC_CM1_2NS || s > SEC_CM4_2NS) throw std::runtime_error("evMap: polynomial not in a cm*_2ns section");
            sec = (uint32_t)s;
            col = (uint32_t)m.sectionPos;
            dim = (uint32_t)m.dim;
        }
        ev_.insert(ev_.end(), {sec, col, dim, e.prime ? 1u : 0u});
    }
    // stage-2 / stage-3 committed polynomials in cm_n order (starks.cpp:14,
    // 406-520): h1/h2 of each plookup, then the Z of each pu, pe, ci context
    auto tmp_col = [&](uint64_t expId, uint32_t &dim) {
        const VarPolMapJ &m = pol(si, exp_pol(si, expId, "ctx"), "ctx");
        if (m.section != S_TMPEXP_N) throw std::runtime_error("ctx: expression not in tmpExp_n");
        dim = (uint32_t)m.dim;
        return (uint32_t)m.sectionPos;
    };
    auto cm_col = [&](uint64_t k, ESection want) {
        if (k >= si.cm_n.size()) throw std::runtime_error("ctx: committed polynomial index out of range");
        const VarPolMapJ &m = pol(si, si.cm_n[k], "ctx");
        if (m.section != want) throw std::runtime_error(std::string("ctx: committed polynomial not in ") + SECTION_NAMES[want]);
        return (uint32_t)m.sectionPos;
    };
    uint64_t nc = si.nCm1;
    for (size_t i = 0; i < si.puCtx.size(); i++) {
        uint32_t df, dt;
        const uint32_t f = tmp_col(si.puCtx[i].fExpId, df), t = tmp_col(si.puCtx[i].tExpId, dt);
        if (df != dt) throw std::runtime_error("puCtx: f and t dimensions differ");
        pu_.insert(pu_.end(), {f, t, cm_col(nc + 2 * i, S_CM2_N), cm_col(nc + 2 * i + 1, S_CM2_N), df});
    }
    nc += 2 * si.puCtx.size();
    auto z_triple = [&](uint64_t numId, uint64_t denId, uint64_t k) {
        uint32_t dn, dd;
        const uint32_t num = tmp_col(numId, dn), den = tmp_col(denId, dd);
        if (dn != 3 || dd != 3) throw std::runtime_error("grand product: num / den must be F_p^3 expressions");
        zctx_.insert(zctx_.end(), {num, den, cm_col(k, S_CM3_N)});
    };
    for (size_t i = 0; i < si.puCtx.size(); i++) z_triple(si.puCtx[i].numId, si.puCtx[i].denId, nc + i);
    nc += si.puCtx.size();
    for (size_t i = 0; i < si.peCtx.size(); i++) z_triple(si.peCtx[i].numId, si.peCtx[i].denId, nc + i);
    nc += si.peCtx.size();
    for (size_t i = 0; i < si.ciCtx.size(); i++) z_triple(si.ciCtx[i].numId, si.ciCtx[i].denId, nc + i);
    info_.n_ev = (uint32_t)si.evMap.size();
    info_.ev = ev_.data();
    info_.n_pu = (uint32_t)si.puCtx.size();
    info_.pu = pu_.data();
    info_.n_zctx = (uint32_t)(zctx_.size() / 3);
    info_.zctx = zctx_.data();
    // the step code (Steps::step2prev ... step52ns, starks.cpp:73-377)
    progs_["step2prev"] = step_to_zxp(si, si.step2prev, false, "step2prev");
    progs_["step3prev"] = step_to_zxp(si, si.step3prev, false, "step3prev");
    progs_["step3"] = step_to_zxp(si, si.step3, false, "step3");
    progs_["step42ns"] = step_to_zxp(si, si.step42ns, true, "step42ns");
    progs_["step52ns"] = step_to_zxp(si, si.step52ns, true, "step52ns");
    info_.step2 = progs_["step2prev"].view();
    info_.step3prev = progs_["step3prev"].view();
    info_.step3 = progs_["step3"].view();
    info_.step42ns = progs_["step42ns"].view();
    info_.step52ns = progs_["step52ns"].view();
    // constants and the committed trace come from files (set_const / set_cm1):
    // no synthetic columns, L_first slot 0 of the placeholder constants
    info_.l_first = 0;
}

const ZxpProgram &ProverInfo::program(const std::string &name) const
{
    auto it = progs_.find(name);
    if (it == progs_.end()) throw std::runtime_error("no program " + name);
    return it->second;
}

json::Value ProverInfo::to_json() const
{
    using json::Value;
    Value j = Value::object();
    auto arr = [](const uint32_t *p, size_t n) {
        Value a = Value::array();
        for (size_t i = 0; i < n; i++) a.push(Value::num(p[i]));
        return a;
    };
    j.set("nBits", Value::num(info_.n_bits));
    j.set("nBitsExt", Value::num(info_.n_bits_ext));
    j.set("nQueries", Value::num(info_.n_queries));
    j.set("friSteps", arr(info_.fri_steps, info_.n_fri_steps));
    j.set("nCm1", Value::num(info_.n_cm1));
    j.set("nCm2", Value::num(info_.n_cm2));
    j.set("nCm3", Value::num(info_.n_cm3));
    j.set("nCm4", Value::num(info_.n_cm4));
    j.set("nTmp", Value::num(info_.n_tmp));
    j.set("nConst", Value::num(info_.n_const));
    j.set("nPublics", Value::num(info_.n_publics));
    j.set("qDeg", Value::num(info_.q_deg));
    j.set("evMap", arr(ev_.data(), ev_.size()));
    j.set("zCtx", arr(zctx_.data(), zctx_.size()));
    j.set("puCtx", arr(pu_.data(), pu_.size()));
    Value ps = Value::object();
    for (const auto &kv : progs_) {
        Value p = Value::object();
        Value ins = Value::array(), opn = Value::array();
        for (const zxp_instr &i : kv.second.instr) ins.push(arr(&i.op, 4));
        for (const zxp_operand &o : kv.second.opnd) opn.push(arr(&o.kind, 4));
        p.set("instr", ins);
        p.set("opnd", opn);
        p.set("nTmp1", Value::num(kv.second.n_tmp1));
        p.set("nTmp3", Value::num(kv.second.n_tmp3));
        ps.set(kv.first, p);
    }
    j.set("programs", ps);
    return j;
}

}  // namespace zkgpu
