"""Column-sharded commit (zkgpu/sharded.py) across processes.

CPU (gloo, world sizes 2 and 4): the distributed logic -- column split, the
all-to-all column->row exchange, per-rank subtrees, sub-root gather, top
levels, openings -- with oracle-backed CPU kernels injected; the root equals
the oracle's single-process tree of the whole LDE and every opening verifies.
GPU (one process, world 1): the same class on the HIP kernels vs the oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class OracleKernels:
    """CPU stand-ins (test infrastructure only) with the GpuKernels interface."""

    def __init__(self, oc):
        self.oc = oc

    def empty(self, shape):
        return torch.zeros(shape, dtype=torch.int64)

    def extend(self, out, src, n, ne, ncols):
        if not ncols:
            return
        x = src[:ncols].numpy().view(np.uint64).T.copy()
        out[:ncols] = torch.from_numpy(np.ascontiguousarray(self.oc.extend_pol(x, ne).T).view(np.int64))

    def merkle(self, src, ld, ncols, nrows):
        rows = np.ascontiguousarray(src[:ncols, :nrows].numpy().view(np.uint64).T)
        return torch.from_numpy(self.oc.merkletree(rows).view(np.int64))

    def root(self, nodes):
        return nodes[-4:].numpy().view(np.uint64).copy()

    def open(self, nodes, src, ld, ncols, nrows, idx):
        rows = np.ascontiguousarray(src[:ncols, :nrows].numpy().view(np.uint64).T)
        nd = nodes.numpy().view(np.uint64)
        out_v, out_s = [], []
        for i in idx:
            v, s = self.oc.merkle_group_proof(nd, rows, int(i))
            out_v.append(v)
            out_s.append(s)
        return np.array(out_v), np.array(out_s)

    def hash_node(self, left, right):
        x = np.zeros(12, np.uint64)
        x[:4], x[4:8] = left, right
        return self.oc.poseidon_hash(x)

    def synchronize(self):
        pass


def _trace(n_bits, ncols, seed=7):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 2**63, size=(ncols, 1 << n_bits), dtype=np.uint64)


def _worker(rank, world, port, n_bits, blow, ncols, q):
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root_dir, os.path.join(root_dir, "zkevm-prover_amd")]
    from oracle import oracle as oc
    from zkgpu.sharded import ShardedCommit, col_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = _trace(n_bits, ncols)
        lo, hi = col_range(ncols, world, rank)
        sc = ShardedCommit(n_bits, blow, ncols, kernels=OracleKernels(oc))
        root = sc.commit(torch.from_numpy(full[lo:hi].view(np.int64).copy()))
        ne = 1 << (n_bits + blow)
        openings = {}
        for idx in (0, 1, ne // 2 - 1, ne // 2, ne - 1, 12345 % ne):
            r = sc.open_local(idx)
            if r is not None:
                openings[idx] = (r[0].tolist(), r[1].tolist())
        q.put((rank, root.tolist(), openings))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,ncols", [(2, 7), (4, 10)])
def test_sharded_commit_gloo(oracle, world, ncols):
    n_bits, blow = 10, 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_bits, blow, ncols, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = _trace(n_bits, ncols)
    lde = oracle.extend_pol(np.ascontiguousarray(full.T), 1 << (n_bits + blow))
    nodes = oracle.merkletree(lde)
    want = [int(v) for v in nodes[-4:]]
    seen = {}
    for rank, root, openings in res:
        assert root == want, rank
        for idx, (vals, sibs) in openings.items():
            assert idx not in seen
            seen[idx] = True
            assert vals == [int(v) for v in lde[idx]]
            assert [int(v) for v in oracle.merkle_root_from_proof(np.array(vals, np.uint64),
                                                                  np.array(sibs, np.uint64), idx)] == want
    assert len(seen) == 6


@pytest.mark.gpu
def test_sharded_commit_gpu_single_rank(oracle, zkgpu):
    """World 1 on the GPU kernels: root and openings vs the oracle."""
    from zkgpu.sharded import ShardedCommit
    n_bits, blow, ncols = 12, 1, 9
    full = _trace(n_bits, ncols, seed=3)
    sc = ShardedCommit(n_bits, blow, ncols, device="cuda:0")
    root = sc.commit(zkgpu.to_device(full))
    lde = oracle.extend_pol(np.ascontiguousarray(full.T), 1 << (n_bits + blow))
    nodes = oracle.merkletree(lde)
    assert np.array_equal(root, nodes[-4:])
    for idx in (0, 77, (1 << (n_bits + blow)) - 1):
        vals, sibs = sc.open_local(idx)
        assert np.array_equal(vals, lde[idx])
        assert np.array_equal(oracle.merkle_root_from_proof(vals, sibs, idx), nodes[-4:])
