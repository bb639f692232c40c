"""The proofs bench.py times, checked at their timed size by a verifier's
replay (tests/stark_verify.py; VERDICT r5 "next" 1-2): no oracle fixture fits
the build container above 2^20 rows for the zkEVM-shaped instance, so the
GPU's proof is re-derived instead -- transcript and query indices, every
Merkle path of the five stage / constant trees and of every FRI layer, every
fold down to finalPol, and the FRI polynomial (step52ns, starks.cpp:371) at
every query row from the opened values (the oracle's interpreter) against
FRI layer 1; for config-4, whose step52ns is the real FRI polynomial, also the
degree of finalPol.

* the zkEVM-shaped instance (fork-9 widths + the five zkEVM-shaped programs,
  bench.stark_instance(.., "zkevm")) at 2^22 (resident plan) and at 2^23 --
  the north-star size: 386 GB resident, so the prover takes the lean plan on
  one MI355X (include/zkgpu_stark.h ZKGPU_MEM_LEAN);
* the config-4 headline instance at 2^23 (also bit-exact against its oracle
  fixture, tests/test_gpu_full_parity.py).
A proof with one opened value changed, or one eval changed, must fail."""
import json

import pytest

pytestmark = pytest.mark.gpu


def _prove(bits, kind, expect_mode):
    import torch
    import bench
    from zkgpu.stark import GpuStark
    torch.cuda.empty_cache()
    inst = bench.stark_instance(bits, 1, 100, 128, kind)
    g = GpuStark(inst)
    try:
        assert g.memory_mode() == expect_mode
        g.witness()
        proof = g.prove()
        return inst, proof, g.verkey(), g.publics()
    finally:
        g.close()


@pytest.mark.parametrize("bits,kind,mode", [(22, "zkevm", "resident"), (23, "zkevm", "lean"), (23, False, "resident")],
                         ids=["zkevm_shaped_2p22", "zkevm_shaped_2p23_lean", "config4_2p23"])
def test_timed_proof_verifies(zkgpu, oracle, bits, kind, mode):
    import stark_verify as sv
    inst, proof, verkey, publics = _prove(bits, kind, mode)
    low = kind is False
    bad = sv.verify(inst, proof, verkey, publics, low_degree=low)
    assert bad["queries"] == 128 and bad["checked"] > 0
    assert not sv.failures(bad), bad
    # a changed opening of the cm1 tree fails its Merkle path
    p2 = json.loads(json.dumps(proof))
    p2["s0_vals1"][5][7] = str((int(p2["s0_vals1"][5][7]) + 1) % sv.P)
    f = sv.failures(sv.verify(inst, p2, verkey, publics, low_degree=low))
    assert f.get("s0") == 1, f
    # a changed eval changes the transcript (other queries) and f at every row
    p3 = json.loads(json.dumps(proof))
    p3["evals"][3][1] = str((int(p3["evals"][3][1]) + 1) % sv.P)
    f = sv.failures(sv.verify(inst, p3, verkey, publics, low_degree=low))
    assert f.get("fri_pol", 0) > 100, f
