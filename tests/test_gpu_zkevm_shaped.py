"""The zkEVM-shaped proof: the fork-9 widths with the five
zkEVM-shaped expression programs (zkgpu/zkevm_shaped.py) -- step2prev /
step3prev / step3 in the n-domain stage slots, step42ns (20 K ops) and
step52ns (1,972 evaluations) on the extended domain, converted from
reference-format bytecode by the product converter -- proved on the GPU and
compared bit for bit with the oracle's proof (starks.cpp:73,155,193,241,371).
The random constraints do not vanish on the trace, so the proof does not
verify; it is deterministic, and every field of it must match."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zkevm_case(oracle):
    from oracle.stark_prover import OracleStark
    from zkgpu.zkevm_shaped import ZkevmShapedStark
    inst = ZkevmShapedStark.create(n_bits=10, n_queries=8)
    o = OracleStark(inst)
    o.witness()
    return inst, o.prove()


def _prove(inst, comm=None):
    from zkgpu.stark import GpuStark
    g = GpuStark(inst, comm=comm)
    g.witness()
    got = g.prove()
    t = g.timers()
    g.close()
    return got, t


@pytest.mark.parametrize("jit", ["0", "2"], ids=["interpreter", "compiled"])
def test_zkevm_shaped_proof_bit_exact(zkgpu, zkevm_case, monkeypatch, jit):
    """interpreter (the 2^10 default) and the compiled segment kernels that
    run at 2^22-2^24 (code objects prebuilt by tools/jit_prebuild.py)"""
    monkeypatch.setenv("ZKGPU_ZXP_JIT", jit)
    inst, ref = zkevm_case
    got, _ = _prove(inst)
    for k in ref:
        assert got[k] == ref[k], k


@pytest.mark.parametrize("jit", ["0", "2"], ids=["interpreter", "compiled"])
def test_zkevm_shaped_repeat_is_deterministic(zkgpu, zkevm_case, monkeypatch, jit):
    """a second proof by the same prover object (the bench's timed loop)
    equals the first: nothing reads a column left over from the last proof.
    Compiled: from the second evaluation of a segmented program on, its
    segments are launched as they are prepared (csrc/zxp_jit.hip
    zxp_jit_run, per-segment staging), so this checks that path too."""
    from zkgpu.stark import GpuStark
    monkeypatch.setenv("ZKGPU_ZXP_JIT", jit)
    inst, ref = zkevm_case
    g = GpuStark(inst)
    g.witness()
    a = g.prove()
    b = g.prove()
    g.close()
    for k in ref:
        assert a[k] == ref[k] and b[k] == ref[k], k
