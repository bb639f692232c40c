"""Multi-process paths on the CPU (no GPU).

* host/comm_host.hpp -- the shared-memory zkgpu_comm the row-sharded prover
  (host/sharded_starks.hpp) exchanges through when its ranks share a machine
  without RCCL peers -- in W = 2 / 4 / 8 forked processes
  (tests/cpp/comm_host_check.cpp): the prover's exchange patterns byte for
  byte, and a failure raised in exchange k + 1 by a fast rank while a slow
  rank still reads exchange k's flag (VERDICT/ADVICE r3: a sticky flag failed
  exchange k on the slow rank and hung the fast one).
* bench.py's multi-rank timing over a gloo process group (world 2): every
  rank reports the max over ranks, as the driver's N > 1 runs need.
"""
import os
import socket
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "comm_host_check")


@pytest.fixture(scope="module")
def comm_check():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-Wall", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-o", BIN, os.path.join(ROOT, "tests", "cpp", "comm_host_check.cpp"),
                           "-lrt"])
    return BIN


@pytest.mark.parametrize("world", [2, 4, 8])
def test_host_exchange_multiprocess(comm_check, world):
    r = subprocess.run([comm_check, str(world)], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_rank(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        got = bench.max_over_ranks(0.25 * (rank + 1), world, dist, torch, "cpu")
        q.put((rank, got, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_bench_max_over_ranks_gloo():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_bench_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=120) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(e is None for *_, e in res), res
    assert all(got == 0.5 for _, got, _ in res), res
