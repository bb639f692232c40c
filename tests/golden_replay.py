"""Replay of the reference's golden recursion proofs (test infrastructure).

Given one zkin proof JSON written by the reference (proof2zkinStark.cpp:8-82
layout) and its verkey, re-derive with a pluggable backend (the CPU oracle, or
the GPU product for parity) everything a verifier can re-derive without the
circuit:
  * the Fiat-Shamir transcript of Starks::genProof (starks.cpp:28-29, 60, 68-69,
    141, 150-151, 222, 234, 293, 306, 336-342) and FRIProve::prove
    (friProve.cpp:30, 125, 130-133), then getPermutations (friProve.cpp:156);
  * every Merkle opening (s0 trees 1/3/4/C and FRI trees s1..s4);
  * every FRI fold, and the last fold into finalPol.
"""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_meta():
    with open(os.path.join(GOLDEN, "golden_meta.json")) as f:
        return json.load(f)


def load_proof(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def arr(x):
    return np.array([int(v) for v in np.ravel(np.array(x, dtype=object))], dtype=np.uint64)


def transcript_challenges(oc, proof, verkey, publics, steps, n_queries):
    """Return (challenges dict, special_x list, query indices)."""
    t = oc.Transcript()
    t.put(arr(verkey))
    t.put(arr(publics))
    ch = {}
    t.put(arr(proof["root1"]))
    ch[0] = t.get_field()
    ch[1] = t.get_field()
    t.put(arr(proof["root2"]))
    ch[2] = t.get_field()
    ch[3] = t.get_field()
    t.put(arr(proof["root3"]))
    ch[4] = t.get_field()
    t.put(arr(proof["root4"]))
    ch[7] = t.get_field()
    t.put(arr(proof["evals"]))
    ch[5] = t.get_field()
    ch[6] = t.get_field()
    special = []
    for si in range(len(steps)):
        special.append(t.get_field())
        if si < len(steps) - 1:
            t.put(arr(proof["s%d_root" % (si + 1)]))
        else:
            t.put(arr(proof["finalPol"]))
    ys = t.get_permutations(n_queries, steps[0])
    return ch, special, [int(y) for y in ys]


def verify_fri(oc, proof, verkey, publics, steps, n_queries, root_from_proof=None, fold_group=None):
    """Re-derive transcript, openings and folds of a zkin-layout proof.
    Returns (mismatch counters, query indices, challenges)."""
    root_from_proof = root_from_proof or oc.merkle_root_from_proof
    fold_group = fold_group or oc.fri_fold_group
    ch, special, ys = transcript_challenges(oc, proof, verkey, publics, steps, n_queries)
    bad = {"s0": 0, "fri_tree": 0, "fold": 0, "final": 0, "checked": 0}
    s0_trees = [("1", proof["root1"]), ("2", proof["root2"]), ("3", proof["root3"]), ("4", proof["root4"]),
                ("C", verkey)]
    for tag, root in s0_trees:
        key = "s0_vals" + tag
        if key not in proof:
            continue
        for q in range(n_queries):
            r = root_from_proof(arr(proof[key][q]), arr(proof["s0_siblings" + tag][q]), ys[q])
            bad["checked"] += 1
            if not np.array_equal(r, arr(root)):
                bad["s0"] += 1
    shift_inv = oc.gl_inv(7)
    for si in range(1, len(steps)):
        pol_bits = steps[si - 1]
        out_bits = steps[si]
        for q in range(n_queries):
            g = ys[q] % (1 << out_bits)
            vals = arr(proof["s%d_vals" % si][q])
            r = root_from_proof(vals, arr(proof["s%d_siblings" % si][q]), g)
            bad["checked"] += 1
            if not np.array_equal(r, arr(proof["s%d_root" % si])):
                bad["fri_tree"] += 1
            folded = fold_group(vals, g, pol_bits, special[si], shift_inv)
            if si < len(steps) - 1:
                j = g >> steps[si + 1]
                expect = arr(proof["s%d_vals" % (si + 1)][q])[3 * j:3 * j + 3]
                if not np.array_equal(folded, expect):
                    bad["fold"] += 1
            else:
                if not np.array_equal(folded, arr(proof["finalPol"][g])):
                    bad["final"] += 1
        for _ in range(pol_bits - out_bits):
            shift_inv = oc.gl_mul(shift_inv, shift_inv)
    return bad, ys, ch


def check_proof(oc, name, root_from_proof=None, fold_group=None):
    """Replay one golden proof; returns (mismatch counters, query indices)."""
    meta = load_meta()
    proof = load_proof(name)
    verkey = meta[meta["proofs"][name]["verkey"]]
    publics = list(proof["publics"]) + list(meta["recursive2_constRoot"])
    bad, ys, _ = verify_fri(oc, proof, verkey, publics, meta["friSteps"], meta["nQueries"],
                            root_from_proof=root_from_proof, fold_group=fold_group)
    return bad, ys
