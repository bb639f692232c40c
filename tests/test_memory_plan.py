"""Per-GPU HBM plan of the prover (zkgpu_stark_memory_plan, host/starks.cpp
Starks::plan) at the fork-9 zkEVM widths
(commit_pols.hpp:1736-1737: 751 / 168 / 408 / 6 committed columns, 234
constants, 389 tmpExp columns) on the 2^23-row trace of BASELINE configs[4]:
one MI355X (288 GB) cannot hold it, eight row-sharded ranks can.  Host code
only; both create calls enforce the same plan against the device's free HBM."""
import pytest

HBM = 288e9


@pytest.fixture(scope="module")
def plan():
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import memory_plan
    inst = SyntheticStark.fork9(23)
    return {w: memory_plan(inst, w) for w in (0, 1, 2, 4, 8)}


def test_fork9_needs_eight_gpus(plan):
    assert plan[8] <= HBM, plan
    assert plan[0] > HBM and plan[1] > HBM, plan
    # the trace itself (n + 2n domains, 1950 + 1561 columns) dominates
    assert plan[8] > (1950 * 2**23 + 1561 * 2**24) * 8 / 8


def test_plan_falls_with_world(plan):
    assert plan[1] > plan[2] > plan[4] > plan[8]
    # every trace section is divided by W; the replicated parts (q / f / FRI,
    # 2n x 3 each) stay
    assert plan[4] / plan[8] > 1.5


def test_config4_fits_one_gpu():
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import memory_plan
    inst = SyntheticStark(n_bits=23, t=33, m=4, n_free=1, n_queries=128)
    assert memory_plan(inst, 0) < HBM / 2


def test_shift_beyond_block_rejected():
    """step1 reads the tables 11 rows ahead: 8 ranks of 2^6 rows (8-row
    blocks) cannot hold that halo -- refused loudly, not mis-proved."""
    from zkgpu import ZkgpuError
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import memory_plan
    inst = SyntheticStark(n_bits=6, t=2, m=1, n_lookups=2, n_queries=4, fri_steps=[7, 5])
    assert memory_plan(inst, 2) > 0
    with pytest.raises(ZkgpuError, match="row shift 11 exceeds"):
        memory_plan(inst, 8)
