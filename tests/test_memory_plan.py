"""Per-GPU HBM plan of the prover (zkgpu_stark_memory_plan, host/starks.cpp
Starks::plan) at the fork-9 zkEVM widths
(commit_pols.hpp:1736-1737: 751 / 168 / 408 / 6 committed columns, 234
constants, 389 tmpExp columns) on the 2^23-row trace of BASELINE configs[4]:
one MI355X cannot hold every section of both domains (the resident plan), the
lean plan (sections sharing one arena by lifetime, ZKGPU_MEM_LEAN) fits it on
one GPU, eight row-sharded ranks hold it too.  Host code only; both create
calls enforce the same plan against the device's free HBM."""
import pytest

HBM = 309.2e9  # 288 GiB: hipMemGetInfo's total on the MI355X boxes (308.4e9 free after init)


@pytest.fixture(scope="module")
def plan():
    from zkgpu.synthetic import SyntheticStark
    from zkgpu.stark import memory_plan
    inst = SyntheticStark.fork9(23)
    return {w: memory_plan(inst, w) for w in (0, 1, 2, 4, 8)}


def test_fork9_resident_needs_eight_gpus(plan):
    assert plan[8] <= HBM, plan
    assert plan[0] > HBM and plan[1] > HBM, plan
    # the trace itself (n + 2n domains, 1950 + 1561 columns) dominates
    assert plan[8] > (1950 * 2**23 + 1561 * 2**24) * 8 / 8


def test_plan_falls_with_world(plan):
    assert plan[1] > plan[2] > plan[4] > plan[8]
    # every trace section is divided by W; the replicated parts (q / f / FRI,
    # 2n x 3 each) stay
    assert plan[4] / plan[8] > 1.4


def test_fork9_two_ranks_fit_with_small_lde_batches(plan):
    """W = 2 at 2^23: the per-rank plan with the default LDE batches (128
    columns at 2^24 rows) exceeds the free HBM; with the 32-column batches
    create_sharded falls back to (fit_lde_batch) it fits"""
    import zkgpu
    N, NE = 1 << 23, 1 << 24
    ms = (751 + 1) // 2  # the largest column share at W = 2
    L = zkgpu.lib()
    ws_default, ws_32 = L.zkgpu_lde_workspace_bytes(N, NE, ms), L.zkgpu_lde_workspace_bytes(N, NE, 32)
    assert ws_default - ws_32 > 15e9
    assert plan[2] > 308e9 > plan[2] - ws_default + ws_32, (plan[2], ws_default, ws_32)


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


def test_fork9_lean_fits_one_gpu():
    """the north-star instance (fork-9 widths, zkEVM-shaped programs, 2^23)
    under the lean plan: <= 280 GB on one GPU, about a
    third less than the resident plan; at 2^22 as well"""
    import bench
    from zkgpu.stark import memory_plan, MEM_LEAN, MEM_RESIDENT
    for bits in (22, 23):
        inst = bench.stark_instance(bits, 1, 100, 128, "zkevm")
        lean, res = memory_plan(inst, 0, MEM_LEAN), memory_plan(inst, 0, MEM_RESIDENT)
        assert res == memory_plan(inst, 0)
        assert lean < 0.72 * res, (bits, lean, res)
        if bits == 23:
            assert lean <= 280e9 < res, (lean, res)
            # the 2n-domain committed sections (751 + 168 + 408 + 6 + 234
            # columns) + the trees bound it from below
            assert lean > (1567 * 2**24) * 8


def test_lean_plan_refused_when_it_cannot_apply():
    """a quotient program that reads an n-domain section: no lean plan"""
    import copy
    import bench
    from zkgpu import ZkgpuError
    from zkgpu import synthetic as sy
    from zkgpu.stark import memory_plan, MEM_LEAN
    inst = copy.deepcopy(bench.stark_instance(10, 1, 100, 16))
    p = inst.programs["step42ns"]
    a = p.o(sy.COL, sy.SEC_CM2_N, 0, 0)
    p.op(sy.ADD, p.o(sy.TMP1, 0, 0, 0), a, a)
    with pytest.raises(ZkgpuError, match="step42ns reads an n-domain section"):
        memory_plan(inst, 0, MEM_LEAN)
    with pytest.raises(ValueError):
        memory_plan(inst, 2, MEM_LEAN)
