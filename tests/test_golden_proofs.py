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


class _CppTranscriptBackend:
    """The oracle with its Transcript swapped for the product's host
    transcript (zkgpu_transcript_*, the C++ class the GPU prover runs)."""

    def __init__(self, oc):
        import zkgpu.stark as zs
        self._oc = oc
        self.Transcript = zs.Transcript

    def __getattr__(self, name):
        return getattr(self._oc, name)


@pytest.mark.parametrize("name", PROOFS)
def test_golden_proof_replay_cpp_transcript(oracle, name):
    """The C++ host transcript (Transcript::put/getField/getPermutations,
    transcript.cpp:4-88) re-derives the reference's challenges and query
    indices: every opening and fold of the golden proof then checks out."""
    from golden_replay import load_proof, transcript_challenges
    backend = _CppTranscriptBackend(oracle)
    bad, ys = check_proof(backend, name)
    meta = load_meta()
    assert bad == {"s0": 0, "fri_tree": 0, "fold": 0, "final": 0, "checked": 8 * meta["nQueries"]}
    proof = load_proof(name)
    verkey = meta[meta["proofs"][name]["verkey"]]
    publics = list(proof["publics"]) + list(meta["recursive2_constRoot"])
    ch_o, sp_o, ys_o = transcript_challenges(oracle, proof, verkey, publics, meta["friSteps"], meta["nQueries"])
    ch_c, sp_c, ys_c = transcript_challenges(backend, proof, verkey, publics, meta["friSteps"], meta["nQueries"])
    assert ys_c == ys_o == list(ys)
    assert all(np.array_equal(ch_o[k], ch_c[k]) for k in ch_o)
    assert all(np.array_equal(a, b) for a, b in zip(sp_o, sp_c))


def test_cpp_transcript_edge_cases(oracle):
    """Partial absorbs, reads across the 12-element output, getPermutations
    spanning several 63-bit fields, argument errors."""
    import zkgpu.stark as zs
    rng = np.random.default_rng(3)
    for n_put in (0, 1, 7, 8, 9, 23):
        a, b = zs.Transcript(), oracle.Transcript()
        v = rng.integers(0, 2**63, n_put, dtype=np.uint64)
        a.put(v)
        b.put(v)
        for _ in range(5):
            assert np.array_equal(a.get_field(), b.get_field())
        assert [int(x) for x in a.get_permutations(40, 23)] == [int(x) for x in b.get_permutations(40, 23)]
    with pytest.raises(Exception):
        zs.Transcript().get_permutations(4, 64)
