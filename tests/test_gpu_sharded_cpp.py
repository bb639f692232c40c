"""The C++ row-sharded prover (host/sharded_starks.hpp, zkgpu_stark_create_sharded)
on the GPU: every rank's proof equals the oracle's single-process proof bit
for bit.

World 1 runs the sharded code path with no exchange (its own slices are
device copies), with and without an RCCL communicator.  Worlds 2 and 4 run
as 2 / 4 processes on the one GPU of the test box with the host-staged
communicator over gloo (RCCL needs one GPU per rank; the same prover code
issues the same exchanges through either).
"""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

INSTANCES = {
    "lookups": dict(n_bits=7, blowup_bits=1, t=3, m=2, n_free=2, n_lookups=2, n_queries=8),
    "blowup4": dict(n_bits=8, blowup_bits=2, t=4, m=1, n_lookups=1, q_deg=4, n_queries=12),
    # the fork-9 zkEVM widths (751 / 168 / 408 / 6 committed, 234 constants,
    # 389 tmpExp, two plookups; next-row reads and shifted stores in the
    # n-domain stage programs): BASELINE configs[4]'s shape at 2^10 rows
    "fork9": dict(fork9=True, n_bits=10),
    # the fork-9 widths with the five zkEVM-shaped expression programs in the
    # stage slots (zkgpu/zkevm_shaped.py): configs[4]'s programs
    "zkevm": dict(zkevm=True, n_bits=10),
    # FRI layer 1 + first fold over the ranks (host/sharded_starks.hpp
    # fri_transpose_layer): four layers; and a first reduction of 4 (kk = 4),
    # which splits over 2 / 4 ranks but not over 8 (the replicated fold)
    "fri4": dict(n_bits=10, t=3, m=2, n_free=2, n_lookups=1, n_queries=8, fri_steps=[11, 7, 4, 2]),
    "fri_kk4": dict(n_bits=9, t=3, m=1, n_lookups=1, n_queries=8, fri_steps=[10, 8, 5]),
}


def _inst(name):
    from zkgpu.synthetic import SyntheticStark
    a = dict(INSTANCES[name])
    if a.pop("zkevm", False):
        from zkgpu.zkevm_shaped import ZkevmShapedStark
        return ZkevmShapedStark.create(**a)
    if a.pop("fork9", False):
        return SyntheticStark.fork9(**a)
    return SyntheticStark(**a)


def _oracle_json(inst):
    from oracle.stark_prover import OracleStark
    o = OracleStark(inst)
    o.witness()
    return o.prove()


@pytest.fixture(scope="module")
def oracle_proofs(oracle):
    return {k: _oracle_json(_inst(k)) for k in INSTANCES}


def _assert_same(got, want):
    for k in want:
        assert got[k] == want[k], k


def test_fork9_single_gpu_equals_oracle(zkgpu, oracle_proofs):
    """the unsharded prover at the fork-9 widths"""
    from zkgpu.stark import GpuStark
    g = GpuStark(_inst("fork9"))
    g.witness()
    _assert_same(g.prove(), oracle_proofs["fork9"])
    g.close()


@pytest.mark.parametrize("name", list(INSTANCES))
def test_sharded_world1_equals_oracle(zkgpu, oracle_proofs, name):
    from zkgpu.stark import EXCHANGE, Comm, GpuStark

    class One:
        c = Comm(0, 1, None, EXCHANGE())

    g = GpuStark(_inst(name), comm=One())
    g.witness()
    _assert_same(g.prove(), oracle_proofs[name])
    t = g.timers()
    # one rank: the LDE goes straight into the row block, no exchange
    assert "STARK_TOTAL" in t and "STARK_STEP_1_LDE" in t and not any("EXCHANGE" in k for k in t)
    g.close()


def test_sharded_world1_rccl(zkgpu, oracle_proofs):
    from zkgpu.stark import GpuStark, RcclComm
    comm = RcclComm()
    g = GpuStark(_inst("lookups"), comm=comm)
    g.witness()
    _assert_same(g.prove(), oracle_proofs["lookups"])
    g.close()
    comm.close()


def test_sharded_rejects_bad_world(zkgpu):
    from zkgpu import ZkgpuError
    from zkgpu.stark import EXCHANGE, Comm, GpuStark

    class Three:
        c = Comm(0, 3, None, EXCHANGE())

    with pytest.raises(ZkgpuError, match="power of two"):
        GpuStark(_inst("lookups"), comm=Three())


def _worker(rank, world, port, q, name, shm, rows=False, env=None):
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root_dir, os.path.join(root_dir, "zkevm-prover_amd"), os.path.join(root_dir, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **(env or {}))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import zkgpu
        from zkgpu.stark import GpuStark, HostStagedComm, ShmComm
        zkgpu.init(0)
        comm = ShmComm(shm, world, rank) if shm else HostStagedComm()
        g = GpuStark(_inst(name), comm=comm)
        if rows == "async":  # trace A, then B queued in the background during A's proof
            a, b = _two_traces(name)
            g.set_cm1(a)
            g.set_cm1_async(b)
            proof = (g.prove(), g.prove())
        elif rows == "missing":  # an f value outside its table: every rank must fail, naming the row
            from oracle.stark_prover import OracleStark
            o = OracleStark(_inst(name))
            o.witness()
            r = o.S[0].copy()
            r[9, _inst(name).cm1_lk[2]] = 12345
            g.set_cm1(r)
            proof = g.prove()
        elif rows:  # the executor's row-major cm1 (each rank takes its rows + halo)
            from oracle.stark_prover import OracleStark
            o = OracleStark(_inst(name))
            o.witness()
            g.set_cm1(o.S[0])
            proof = g.prove()
        else:
            g.witness()
            proof = g.prove()
        q.put((rank, proof, g.timers(), None))
        g.close()
        comm.close()
    except Exception:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _two_traces(name):
    """the instance's witness and a second trace differing in its free
    (unconstrained) cm1 columns"""
    import numpy as np
    from oracle.stark_prover import OracleStark
    inst = _inst(name)
    o = OracleStark(inst)
    o.witness()
    a = o.S[0].copy()
    free = list(range(3 * inst.t, 3 * inst.t + inst.n_free))
    b = a.copy()
    b[:, free] = np.random.default_rng(1).integers(0, 2**63, size=(b.shape[0], len(free)), dtype=np.uint64)
    return a, b


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,name,comm", [(2, "lookups", "gloo"), (4, "lookups", "gloo"), (2, "blowup4", "gloo"),
                                             (2, "lookups", "shm"), (4, "blowup4", "shm"), (8, "lookups", "shm"),
                                             (2, "fork9", "gloo"), (8, "fork9", "shm"), (4, "lookups", "shm-rows"),
                                             (2, "zkevm", "shm"), (8, "zkevm", "shm"), (2, "fri4", "shm"),
                                             (8, "fri4", "shm"), (4, "fri_kk4", "shm"), (8, "fri_kk4", "shm")])
def test_sharded_multiprocess_equals_oracle(oracle_proofs, world, name, comm):
    """gloo = HostStagedComm (Python, torch.distributed); shm = ShmComm
    (host/comm_host.hpp, shared memory + process-shared barriers); -rows: the
    trace handed over as the executor's row-major buffer (set_cm1)"""
    import multiprocessing as mp
    import uuid
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    shm = "/zkgpu_t_%s" % uuid.uuid4().hex[:12] if comm.startswith("shm") else None
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, name, shm, comm.endswith("-rows")))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errs = [e for *_, e in res if e]
    assert not errs, errs[0]
    for _, proof, timers, _ in res:
        _assert_same(proof, oracle_proofs[name])
        assert timers["STARK_STEP_1_EXCHANGE"] >= 0
        # packed exchanges: one message per peer and direction, whatever the
        # column count (the commits of fork-9's 751 columns included)
        assert 0 < timers["COUNT_COMM_MAX_OPS"] <= 2 * (world - 1), timers["COUNT_COMM_MAX_OPS"]
        # the communicator's world and this proof's exchange volume
        assert timers["COUNT_COMM_WORLD"] == world
        assert timers["COUNT_COMM_EXCHANGES"] > 0
        assert timers["COUNT_COMM_BYTES_SENT"] >= timers["COUNT_COMM_MAX_BYTES_SENT"] > 0


@pytest.mark.parametrize("world", [4, 8])
def test_sharded_set_cm1_async(oracle, world):
    """Back-to-back sharded proofs with the next trace queued in the
    background (set_cm1_async: each rank loads its rows [r0, r0 + ldn) mod N,
    the last rank's in two pieces across the domain end): both proofs equal
    the oracle's proofs of their traces."""
    import multiprocessing as mp
    import uuid
    from oracle.stark_prover import OracleStark
    a, b = _two_traces("lookups")
    want = []
    for t in (a, b):
        o = OracleStark(_inst("lookups"))
        o.witness()
        o.S[0][:] = t
        want.append(o.prove())
    assert want[0] != want[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    shm = "/zkgpu_t_%s" % uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "lookups", shm, "async")) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errs = [e for *_, e in res if e]
    assert not errs, errs[0]
    for _, (pa, pb), _, _ in res:
        _assert_same(pa, want[0])
        _assert_same(pb, want[1])


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_lookup_value_not_in_table(oracle, world):
    """calculateH1H2 over the ranks (h1h2_sharded): an f value that is in no
    table row stops EVERY rank with the reference's error and the f row
    (polinomial.hpp:409-413), as on one GPU (test_gpu_stark.py)"""
    import multiprocessing as mp
    import uuid
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    shm = "/zkgpu_t_%s" % uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "lookups", shm, "missing")) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for _, proof, _, err in res:
        assert proof is None and err and "Number not included: w=9" in err, err


@pytest.mark.parametrize("world,k", [(2, 2), (2, 9), (4, 14), (2, 30)])
def test_sharded_rank_failure_releases_peers(oracle, world, k):
    """A rank that fails locally in the middle of a sharded proof (injected
    before its k-th exchange: setup, the commits, calculateH1H2's five
    exchanges, the quotient, FRI) aborts the communicator (zkgpu_comm.abort,
    ShardedStarks::abort_comm): every other rank's next exchange fails at once
    instead of waiting for it (h1h2_sharded's local errors left the
    peers in the collective).  No rank may hang: all report within seconds,
    well inside the 20 s exchange deadline."""
    import multiprocessing as mp
    import uuid
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    shm = "/zkgpu_t_%s" % uuid.uuid4().hex[:12]
    env = {"ZKGPU_TEST_FAIL_EXCHANGE": "%d:%d" % (world - 1, k), "ZKGPU_COMM_TIMEOUT_S": "20"}
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "lookups", shm, False, env)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errs = {r: e for r, proof, _, e in res}
    assert all(errs[r] for r in range(world)), errs
    assert "injected failure before exchange %d" % k in errs[world - 1], errs[world - 1]
    for r in range(world - 1):
        assert "a rank aborted" in errs[r] or "aborted or timed out" in errs[r], errs[r]
