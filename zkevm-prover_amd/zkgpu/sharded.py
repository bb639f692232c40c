"""Column-sharded commit of one trace across the GPUs of a node
(BASELINE.json configs[4]).

One process per GPU.  The committed section of a stage (n rows x C columns,
e.g. cm1: 2^23 x 100) is split by COLUMNS: rank r owns the contiguous columns
[col_lo(r), col_hi(r)).  One commit (the LDE + merkelize of
Starks::genProof stage k, starks.cpp:53-57) is then:

  1. LDE of the owned columns on the owning GPU (columns are independent:
     NTT_Goldilocks::extendPol per column, no communication);
  2. the only exchange: an all-to-all (RCCL over xGMI) that turns column
     blocks into ROW blocks -- rank r receives rows
     [r NE/W, (r+1) NE/W) of every column, already column-major with
     ld = NE/W, which is the layout the Merkle kernel reads;
  3. each GPU merkelizes its row block: a power-of-two block of leaves is an
     exact subtree of the full tree (merkleTreeGL.cpp:37-44 layout);
  4. all-gather of the W sub-roots (32 B each) and the top log2(W) levels,
     hashed on every rank -> the root, identical to the single-GPU root.
Openings (MerkleTreeGL::getGroupProof, merkleTreeGL.cpp:12-35) are served by
the rank that owns the row block: row values + subtree siblings, then the
top-level siblings from the gathered sub-roots.

The kernels are pluggable so the distributed logic is testable on CPU with
gloo (tests inject CPU kernels); the default is the GPU (libzkgpu) and there
is no CPU fallback in the product.
"""
import numpy as np


def _staged(group, t):
    """gloo cannot run collectives on device tensors: stage through the host
    (tests of the multi-process path on one GPU); RCCL ("nccl") runs on device."""
    import torch.distributed as dist
    try:
        backend = dist.get_backend(group)
    except Exception:
        backend = "gloo"
    return backend != "nccl" and t.is_cuda


def all_gather(t, group=None):
    """List of every rank's tensor (same shape), on t's device."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [t]
    stage = _staged(group, t)
    src = t.cpu() if stage else t.contiguous()
    out = [torch.empty_like(src) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, src, group=group)
    return [o.to(t.device) for o in out] if stage else out


def all_to_all(out, inp, out_splits, in_splits, group=None):
    """all_to_all_single over flat tensors (RCCL on device; gloo via the host)."""
    import torch.distributed as dist
    if _staged(group, inp):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def col_range(ncols, world, rank):
    """Balanced contiguous column split."""
    base, extra = divmod(ncols, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class GpuKernels:
    """libzkgpu kernels on the current torch device (column-major tensors)."""

    def __init__(self, device):
        import torch
        import zkgpu
        self.torch, self.zk, self.device = torch, zkgpu, device

    def empty(self, shape):
        return self.torch.empty(shape, dtype=self.torch.int64, device=self.device)

    def extend(self, out, src, n, ne, ncols):
        if ncols:
            self.zk.extend_pol_dev(out, ne, src, n, ne, n, ncols)

    def merkle(self, src, ld, ncols, nrows):
        nodes = self.empty(self.zk.merkle_num_elements(nrows))
        self.zk.merkletree_dev(nodes, src, ld, ncols, nrows)
        return nodes

    def root(self, nodes):
        return self.zk.from_device(nodes[-4:]).copy()

    def open(self, nodes, src, ld, ncols, nrows, idx):
        return self.zk.merkle_open_dev(nodes, src, ld, ncols, nrows, np.asarray(idx, np.uint64))

    def hash_node(self, left, right):
        x = np.zeros(12, np.uint64)
        x[:4], x[4:8] = left, right
        return self.zk.poseidon_hash(x)

    def synchronize(self):
        self.torch.cuda.synchronize()


class ShardedCommit:
    """Commit one n-row trace of ncols columns, column-sharded over the
    process group; `kernels` defaults to the GPU."""

    def __init__(self, n_bits, blowup_bits, ncols, group=None, kernels=None, device=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n = 1 << n_bits
        self.ne = 1 << (n_bits + blowup_bits)
        if self.ne % self.world or (self.world & (self.world - 1)):
            raise ValueError("world size must be a power of two dividing the extended domain")
        self.rows = self.ne // self.world  # row block per rank after the exchange
        self.ncols = ncols
        self.lo, self.hi = col_range(ncols, self.world, self.rank)
        self.k = kernels if kernels is not None else GpuKernels(device)
        self.counts = [col_range(ncols, self.world, r)[1] - col_range(ncols, self.world, r)[0]
                       for r in range(self.world)]
        self.nodes = None
        self.block = None
        self.top = None

    def commit(self, local_cols):
        """local_cols: (hi - lo) x n column-major tensor of the owned columns.
        Returns the root (4 u64, identical on every rank)."""
        k, W, rows = self.k, self.world, self.rows
        c_r = self.hi - self.lo
        ext = k.empty((max(c_r, 1), self.ne))
        k.extend(ext, local_cols, self.n, self.ne, c_r)
        if W == 1:
            self.block = ext
        else:
            # pack [dest rank][owned column][row in block] (contiguous per destination)
            send = ext[:c_r].reshape(c_r, W, rows).permute(1, 0, 2).contiguous().reshape(-1)
            self.block = k.empty((self.ncols, rows))
            all_to_all(self.block.reshape(-1), send, [c * rows for c in self.counts], [c_r * rows] * W,
                       group=self.group)
        return self._merkelize()

    def commit_rows(self, block):
        """Commit when every rank already holds its row block of the extended
        evaluations (ncols x rows, column-major): subtree + sub-root gather."""
        self.block = block
        return self._merkelize()

    def _merkelize(self):
        k, W, rows = self.k, self.world, self.rows
        self.nodes = k.merkle(self.block, rows, self.ncols, rows)
        sub = k.root(self.nodes)
        if W == 1:
            self.top = [[sub]]
            return sub
        import torch
        mine = torch.from_numpy(sub.view(np.int64).copy())
        if self._backend_is_nccl():
            mine = mine.to(self.block.device)
        gathered = all_gather(mine, self.group)
        level = [g.cpu().numpy().view(np.uint64).copy() for g in gathered]
        self.top = [level]
        while len(level) > 1:
            level = [k.hash_node(level[2 * i], level[2 * i + 1]) for i in range(len(level) // 2)]
            self.top.append(level)
        return level[0]

    def _backend_is_nccl(self):
        try:
            return self.dist.get_backend(self.group) == "nccl"
        except Exception:
            return False

    def open_local_many(self, idxs):
        """{global row: (values, siblings)} for the rows of idxs this rank owns
        (one batched opening launch)."""
        own = sorted({int(i) for i in idxs if int(i) // self.rows == self.rank})
        if not own:
            return {}
        vals, sibs = self.k.open(self.nodes, self.block, self.rows, self.ncols, self.rows,
                                 [i % self.rows for i in own])
        out = {}
        for n, idx in enumerate(own):
            top_sibs = []
            j = self.rank
            for level in self.top[:-1]:
                top_sibs.append(level[j ^ 1])
                j >>= 1
            out[idx] = (vals[n], np.concatenate([sibs[n].reshape(-1, 4),
                                                 np.array(top_sibs, np.uint64).reshape(-1, 4)]))
        return out

    def open_local(self, idx):
        """Opening of global row idx if this rank owns it: (values, siblings)
        with siblings bottom-up (subtree levels, then top levels); else None."""
        owner, local = divmod(int(idx), self.rows)
        if owner != self.rank:
            return None
        vals, sibs = self.k.open(self.nodes, self.block, self.rows, self.ncols, self.rows, [local])
        top_sibs = []
        j = owner
        for level in self.top[:-1]:
            top_sibs.append(level[j ^ 1])
            j >>= 1
        sibs = np.concatenate([sibs[0].reshape(-1, 4), np.array(top_sibs, np.uint64).reshape(-1, 4)])
        return vals[0], sibs
