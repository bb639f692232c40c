"""The batch-proof driver end to end on the GPU: the reference's input files
(starkinfo JSON, constant polynomials, constant tree, committed trace,
publics) -> zkgpu_batch_prover -> batch_proof.zkin.json byte-identical to the
oracle's proof in proof2zkinStark layout (tests/test_starkinfo.py checks the
loader and writers on the CPU)."""
import json
import os
import subprocess
import uuid

import numpy as np
import pytest

from test_starkinfo import DRIVER

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kw", [dict(n_bits=10, t=4, m=2, n_queries=16),
                                dict(n_bits=9, blowup_bits=2, t=3, m=1, n_lookups=1, q_deg=4, n_queries=12)])
def test_batch_prover_drop_in(oracle, tmp_path, kw):
    import zkgpu.starkinfo as zs
    from oracle.stark_prover import OracleStark
    from zkgpu.synthetic import SyntheticStark
    inst = SyntheticStark(**kw)
    o = OracleStark(inst)
    o.witness()
    proof = o.prove()
    cfg = zs.write_inputs(str(tmp_path), inst, o.S[4], o.S[9], o.const_nodes, o.S[0], o.publics)
    r = subprocess.run([DRIVER, cfg], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = tmp_path / "out"
    assert (out / "batch_proof.zkin.json").read_text() == zs.zkin_text(proof, o.publics, inst.n_cm2, inst.n_cm3)
    full = json.loads((out / "batch_proof.proof.json").read_text())
    assert full["root1"] == proof["root1"] and full["evals"] == proof["evals"]


def test_batch_prover_rejects_wrong_const_tree(oracle, tmp_path):
    """a constant tree whose root is not the tree of the constant file fails loudly"""
    import zkgpu.starkinfo as zs
    from oracle.stark_prover import OracleStark
    from zkgpu.synthetic import SyntheticStark
    inst = SyntheticStark(n_bits=8, t=2, m=1, n_queries=8)
    o = OracleStark(inst)
    o.witness()
    nodes = o.const_nodes.copy()
    nodes[-1] ^= 1
    cfg = zs.write_inputs(str(tmp_path), inst, o.S[4], o.S[9], nodes, o.S[0], o.publics)
    r = subprocess.run([DRIVER, cfg], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "zkevmConstantsTree" in r.stderr, r.stderr
    assert not os.path.exists(tmp_path / "out" / "batch_proof.zkin.json")


def _sharded_run(cfg, world, comm):
    procs = [subprocess.Popen([DRIVER, "--shard", "%d/%d" % (r, world), "--comm", comm, cfg], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=120))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    bad = [(r, p.returncode, err) for r, (p, (_, err)) in enumerate(zip(procs, outs)) if p.returncode != 0]
    assert not bad, "\n".join("rank %d exit %s: %s" % b for b in bad)
    return [err for _, err in outs]


@pytest.mark.parametrize("world,comm,fork9", [(2, "host", False), (4, "host", False), (1, "rccl", False),
                                              (8, "host", True)])
def test_batch_prover_sharded(oracle, tmp_path, world, comm, fork9):
    """--shard r/W: W driver processes prove ONE proof row-sharded
    (zkgpu_stark_create_sharded); rank 0's zkin equals the oracle's.  host =
    shared-memory exchange (the W processes share the one GPU here); rccl at
    world 1 exercises the id file and communicator set-up; fork9: the
    zkEVM's widths (751 / 168 / 408 / 6 committed, 234 constants) from the
    reference's file formats over 8 ranks."""
    import zkgpu.starkinfo as zs
    from oracle.stark_prover import OracleStark
    from zkgpu.synthetic import SyntheticStark
    inst = (SyntheticStark.fork9(n_bits=10, n_queries=8) if fork9 else
            SyntheticStark(n_bits=9, blowup_bits=1, t=4, m=2, n_lookups=1, n_queries=12))
    o = OracleStark(inst)
    o.witness()
    proof = o.prove()
    cfg = zs.write_inputs(str(tmp_path), inst, o.S[4], o.S[9], o.const_nodes, o.S[0], o.publics)
    idf = tmp_path / "rccl.id"
    spec = "host:/zkgpu_t_%s" % uuid.uuid4().hex[:12] if comm == "host" else "rccl:%s" % idf
    if comm == "rccl":  # an id file left at the same path by an earlier run (other tag): overwritten, not used
        idf.write_bytes(b"ZKGPUID1" + (9).to_bytes(4, "little") + b"stale-run" + bytes(128))
    for run in range(2 if comm == "rccl" else 1):  # twice against the same id path
        errs = _sharded_run(cfg, world, spec)
        assert all("[%d/%d]" % (r, world) in e for r, e in enumerate(errs))
        assert (tmp_path / "out" / "batch_proof.zkin.json").read_text() == zs.zkin_text(proof, o.publics, inst.n_cm2,
                                                                                          inst.n_cm3)
        if comm == "rccl":
            assert not idf.exists(), "rank 0 removes the id file once the communicator exists"
