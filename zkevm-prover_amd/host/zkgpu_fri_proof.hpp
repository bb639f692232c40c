// zkgpu_fri_proof.hpp -- the reference's proof objects from the GPU prover's
// flat proof buffer (include/zkgpu_stark.h):
//   proof2json       FRIProof::proofs.proof2json() (fri/friProof.hpp:176-235):
//                    {root1..root4, evals, fri: [tree_0 .. tree_{steps-1}, finalPol]},
//                    tree = {root, polQueries}; tree 0 holds five Merkle
//                    proofs per query (cm1 cm2 cm3 cm4 const), its root is
//                    never set (FRIProve only sets trees[si + 1]) and stays 0
//   proof2zkinStark  fri/proof2zkinStark.cpp:8-82, the same key order
//                    (s0_vals2 / s0_vals3 and their siblings omitted when the
//                    stage has no columns)
// Values are canonical decimal strings (Goldilocks::toString).
#pragma once
#include <stdint.h>

#include <stdexcept>
#include <string>

#include "../../include/zkgpu_stark.h"
#include "zkgpu_json.hpp"

namespace zkgpu {

inline json::Value proof2json(const uint64_t *flat, uint64_t len, const zkgpu_stark_info &in)
{
    using json::Value;
    const uint64_t P = 0xFFFFFFFF00000001ULL;
    uint64_t pos = 0;
    auto next = [&]() {
        if (pos >= len) throw std::runtime_error("proof2json: flat proof too short");
        return Value::str(std::to_string(flat[pos++] % P));
    };
    auto list = [&](uint64_t n) {
        Value a = Value::array();
        for (uint64_t i = 0; i < n; i++) a.push(next());
        return a;
    };
    auto nested = [&](uint64_t rows, uint64_t w) {
        Value a = Value::array();
        for (uint64_t i = 0; i < rows; i++) a.push(list(w));
        return a;
    };
    const uint32_t Q = in.n_queries, S = in.n_fri_steps;
    Value j = Value::object();
    j.set("root1", list(4));
    j.set("root2", list(4));
    j.set("root3", list(4));
    j.set("root4", list(4));
    j.set("evals", nested(in.n_ev, 3));
    // FRI steps 1 .. S-1 (flat order: root, vals, siblings per step)
    std::vector<Value> trees(S);
    for (uint32_t si = 1; si < S; si++) {
        Value t = Value::object();
        t.set("root", list(4));
        const uint64_t w = 3ULL << (in.fri_steps[si - 1] - in.fri_steps[si]);
        std::vector<Value> vals(Q), sibs(Q);
        for (uint32_t q = 0; q < Q; q++) vals[q] = list(w);
        for (uint32_t q = 0; q < Q; q++) sibs[q] = nested(in.fri_steps[si], 4);
        Value pq = Value::array();
        for (uint32_t q = 0; q < Q; q++) {
            Value mp = Value::array();
            mp.push(vals[q]);
            mp.push(sibs[q]);
            pq.push(mp);
        }
        t.set("polQueries", pq);
        trees[si] = t;
    }
    // step 0: values of the five trees, then their siblings
    const uint32_t widths[5] = {in.n_cm1, in.n_cm2, in.n_cm3, in.n_cm4, in.n_const};
    std::vector<std::vector<Value>> v0(5, std::vector<Value>(Q)), s0(5, std::vector<Value>(Q));
    for (int k = 0; k < 5; k++)
        for (uint32_t q = 0; q < Q; q++) v0[k][q] = list(widths[k]);
    for (int k = 0; k < 5; k++)
        for (uint32_t q = 0; q < Q; q++) s0[k][q] = nested(in.n_bits_ext, 4);
    Value t0 = Value::object();
    Value zero = Value::array();
    for (int i = 0; i < 4; i++) zero.push(Value::str("0"));
    t0.set("root", zero);
    Value pq0 = Value::array();
    for (uint32_t q = 0; q < Q; q++) {
        Value e = Value::array();
        for (int k = 0; k < 5; k++) {
            Value mp = Value::array();
            mp.push(v0[k][q]);
            mp.push(s0[k][q]);
            e.push(mp);
        }
        pq0.push(e);
    }
    t0.set("polQueries", pq0);
    trees[0] = t0;
    Value fri = Value::array();
    for (uint32_t si = 0; si < S; si++) fri.push(trees[si]);
    fri.push(nested(1ULL << in.fri_steps[S - 1], 3));
    j.set("fri", fri);
    if (pos != len) throw std::runtime_error("proof2json: flat proof length mismatch");
    return j;
}

// fri/proof2zkinStark.cpp:8-82
inline json::Value proof2zkinStark(const json::Value &proof)
{
    using json::Value;
    Value z = Value::object();
    z.set("root1", proof["root1"]);
    z.set("root2", proof["root2"]);
    z.set("root3", proof["root3"]);
    z.set("root4", proof["root4"]);
    z.set("evals", proof["evals"]);
    const Value &fri = proof["fri"];
    const size_t nq = fri[0]["polQueries"].size();
    for (size_t i = 1; i + 1 < fri.size(); i++) {
        const std::string s = "s" + std::to_string(i);
        z.set(s + "_root", fri[i]["root"]);
        Value vals = Value::array(), sibs = Value::array();
        for (size_t q = 0; q < nq; q++) {
            vals.push(fri[i]["polQueries"][q][0]);
            sibs.push(fri[i]["polQueries"][q][1]);
        }
        z.set(s + "_vals", vals);
        z.set(s + "_siblings", sibs);
    }
    const Value &pq = fri[0]["polQueries"];
    const bool has2 = nq && pq[0][1][0].size(), has3 = nq && pq[0][2][0].size();
    auto col = [&](int k, int part) {
        Value a = Value::array();
        for (size_t q = 0; q < nq; q++) a.push(pq[q][k][part]);
        return a;
    };
    z.set("s0_vals1", col(0, 0));
    if (has2) z.set("s0_vals2", col(1, 0));
    if (has3) z.set("s0_vals3", col(2, 0));
    z.set("s0_vals4", col(3, 0));
    z.set("s0_valsC", col(4, 0));
    z.set("s0_siblings1", col(0, 1));
    if (has2) z.set("s0_siblings2", col(1, 1));
    if (has3) z.set("s0_siblings3", col(2, 1));
    z.set("s0_siblings4", col(3, 1));
    z.set("s0_siblingsC", col(4, 1));
    z.set("finalPol", fri[fri.size() - 1]);
    return z;
}

}  // namespace zkgpu
