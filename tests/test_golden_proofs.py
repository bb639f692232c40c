"""Known-answer tests: the CPU oracle replays the reference's golden proofs.

Pins Poseidon-GL, linear_hash, the Merkle layout and openings, the transcript,
getPermutations, the FRI fold (16/8-point INTTs, shift and root conventions)
and the cubic extension against outputs the reference itself produced
(testvectors/aggregatedProof/recursive1.zkin.proof_0.json and
testvectors/finalProof/recursive2.zkin.proof_01.json, copied to tests/golden/).
"""
import numpy as np
import pytest

from golden_replay import check_proof, load_meta

PROOFS = ["recursive1.zkin.proof_0.json", "recursive2.zkin.proof_01.json"]


@pytest.mark.parametrize("name", PROOFS)
def test_golden_proof_replay(oracle, name):
    bad, ys = check_proof(oracle, name)
    meta = load_meta()
    assert len(ys) == meta["nQueries"]
    assert all(0 <= y < (1 << meta["friSteps"][0]) for y in ys)
    # 4 s0 trees x 43 + 4 FRI trees x 43 openings
    assert bad["checked"] == 8 * meta["nQueries"]
    assert bad == {"s0": 0, "fri_tree": 0, "fold": 0, "final": 0, "checked": bad["checked"]}


def test_empty_stage_root(oracle):
    """root2 of recursive1 commits an empty section (0 columns): the root of
    2^20 all-zero leaf digests (linear_hash width 0)."""
    from golden_replay import load_proof, arr
    proof = load_proof(PROOFS[0])
    h = np.zeros(4, np.uint64)
    for _ in range(20):
        h = oracle.poseidon_hash(np.concatenate([h, h, np.zeros(4, np.uint64)]))
    assert np.array_equal(h, arr(proof["root2"]))
