"""The verifier-side replay (tests/stark_verify.py) pinned on the oracle's
own proofs (CPU): config-4 and the zkEVM-shaped instance at 2^10 pass every
check; a changed opening, FRI value, eval or final-polynomial entry fails the
check that covers it.  The GPU side runs the same replay on the proofs bench.py
times (tests/test_gpu_verify_full.py)."""
import json

import pytest

import stark_verify as sv  # noqa: E402


@pytest.fixture(scope="module", params=[False, "zkevm"], ids=["config4", "zkevm_shaped"])
def proved(request, oracle):
    import bench
    from oracle.stark_prover import OracleStark
    inst = bench.stark_instance(10, 1, 100, 16, request.param)
    o = OracleStark(inst)
    o.witness()
    return inst, o.prove(), o.verkey, o.publics, request.param is False


def _bump(v):
    return str((int(v) + 1) % sv.P)


def test_oracle_proof_verifies(proved):
    inst, proof, vk, pub, low = proved
    bad = sv.verify(inst, proof, vk, pub, low_degree=low)
    assert bad["queries"] == 16 and bad["checked"] == 16 * (5 + len(inst.fri_steps) - 1)
    assert not sv.failures(bad), bad


def test_changed_values_fail(proved):
    inst, proof, vk, pub, low = proved
    for key, path, check in (("s0_vals3", (2, 1), "s0"), ("s1_vals", (4, 0), "fri_tree"),
                             ("evals", (0, 2), "fri_pol"), ("s0_vals4", (0, 0), "s0")):
        p = json.loads(json.dumps(proof))
        p[key][path[0]][path[1]] = _bump(p[key][path[0]][path[1]])
        f = sv.failures(sv.verify(inst, p, vk, pub, low_degree=low))
        assert f.get(check), (key, f)


def test_final_polynomial_degree(proved):
    """config-4's step52ns is the FRI polynomial: finalPol has low degree, and
    a changed finalPol entry breaks it (and the last fold)"""
    inst, proof, vk, pub, low = proved
    if not low:
        pytest.skip("the zkEVM-shaped step52ns is a shape stand-in, not the FRI polynomial (stark_verify doc)")
    from oracle import oracle as oc
    assert sv.final_degree_ok(oc, inst, proof)[0]
    p = json.loads(json.dumps(proof))
    p["finalPol"][3][0] = _bump(p["finalPol"][3][0])
    assert not sv.final_degree_ok(oc, inst, p)[0]


def test_quotient_identity_at_xi(proved):
    """config-4 is a valid AIR: C(xi) Z_H(xi)^-1 == sum_p xi^(pN) q_p(xi) from
    the evals; a changed eval of a constrained column or of a quotient piece
    breaks it"""
    inst, proof, vk, pub, low = proved
    if not low:
        pytest.skip("the zkEVM-shaped trace does not satisfy its stand-in constraints (stark_verify doc)")
    from oracle import oracle as oc
    from zkgpu import synthetic as sy
    steps = list(inst.fri_steps)
    _, _, ch = sv.gr.verify_fri(oc, proof, [int(v) for v in vk], [int(v) for v in pub], steps, inst.n_queries)
    cz, q = sv.quotient_identity(inst, proof, ch, pub)
    assert cz == q and any(q)
    for i in (inst.ev_index[(sy.SEC_CM1_2NS, 2, 0)], inst.ev_index[(sy.SEC_CM4_2NS, 3, 0)]):
        p = json.loads(json.dumps(proof))
        p["evals"][i][1] = _bump(p["evals"][i][1])
        cz, q = sv.quotient_identity(inst, p, ch, pub)
        assert cz != q
        assert sv.failures(sv.verify(inst, p, vk, pub)).get("quotient_at_xi")
