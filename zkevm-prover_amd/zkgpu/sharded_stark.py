"""Row-sharded full STARK proof of ONE trace across the GPUs of a node
(BASELINE.json configs[4]: "the same BatchProof trace
column-sharded across 8 x MI355X with RCCL all-to-all NTT transpose").

One process per GPU, world size W a power of two.  Starks::genProof
(starks.cpp:9-404) with the extended (2n) domain -- where the bytes and the
hashing are -- partitioned by ROWS, and the n-domain stage work replicated:

  setup     constants (n rows) on every rank; the constant tree is a sharded
            commit (below); its root is the verkey.
  commit k  (stages 1-3, starks.cpp:53-57,134-138,215-219) rank r extends its
            column share of the committed section (NTT_Goldilocks::extendPol,
            no communication), ONE all-to-all over xGMI turns column blocks
            into row blocks [r B, (r+1) B) of every column (B = 2n / W), each
            rank hashes its block as an exact subtree and the W sub-roots are
            all-gathered (zkgpu/sharded.py ShardedCommit).  The halo -- the
            first 2^blowup rows of the next block, read by "next row"
            constraints -- is all-gathered (2^blowup x width elements per rank).
  n-domain  step2 / H1H2 / step3prev / calculateZ (starks.cpp:67-211) run on
            every rank over the replicated n-row sections (tens of MB at
            2^23; the extended sections are hundreds of GB at fork-9 widths).
  stage 4   the quotient program (step42ns) on each rank's rows
            (zkgpu_zxp_eval_block_dev: x_i = 7 w^(rB + i), halo rows, no
            wrap); q (2n x 3) is all-gathered, INTT / split / NTT
            (starks.cpp:226-296) run on every rank, each commits its rows.
  stage 5   evmap: each rank sums its rows, partial sums are all-gathered and
            added mod p (starks.cpp:556-669); xDivXSub and the FRI program
            (step52ns) on each rank's rows; f (2n x 3) is all-gathered.
  FRI       folds, layer trees and the final polynomial on every rank
            (friProve.cpp:5-150; 2n x 3 elements, < 1 % of the proof).
  queries   each s0 opening is produced by the rank owning its row
            (subtree siblings + top levels) and all-gathered.
The transcript (transcript.cpp:4-87) runs on every rank on identical inputs,
so every rank derives the same challenges.  The proof equals the
single-process proof bit for bit (tests/test_sharded_stark.py: oracle-backed
CPU kernels over gloo at world sizes 1, 2 and 4, and the HIP kernels).

The kernels are pluggable (GpuStarkKernels by default, HIP through the
libzkgpu C-ABI); there is no CPU fallback in the product.
"""
import numpy as np

from .sharded import GpuKernels, ShardedCommit, all_gather
from .stark import to_json

P = 0xFFFFFFFF00000001
W32 = 7277203076849721926  # Goldilocks::w(32)


def w_of(n_bits):
    w = W32
    for _ in range(n_bits, 32):
        w = w * w % P
    return w


class Transcript:
    """Transcript (transcript.cpp:4-87); hash_full = hash_full_result."""

    def __init__(self, hash_full):
        self.h = hash_full
        self.state = [0] * 4
        self.pending = []
        self.out = [0] * 12
        self.out_cursor = 0

    def _absorb(self):
        x = np.zeros(12, np.uint64)
        x[:len(self.pending)] = self.pending
        x[8:] = self.state
        self.out = [int(v) for v in self.h(x)]
        self.out_cursor = 12
        self.pending = []
        self.state = self.out[:4]

    def put(self, vals):
        for v in np.asarray(vals, np.uint64).reshape(-1):
            self.pending.append(int(v))
            self.out_cursor = 0
            if len(self.pending) == 8:
                self._absorb()

    def get_fields1(self):
        if self.out_cursor == 0:
            self._absorb()
        r = self.out[(12 - self.out_cursor) % 12]
        self.out_cursor -= 1
        return r

    def get_field(self):
        return np.array([self.get_fields1() for _ in range(3)], np.uint64)

    def get_permutations(self, n, nbits):
        nfields = (n * nbits - 1) // 63 + 1
        f = [self.get_fields1() % P for _ in range(nfields)]
        res, cf, cb = [], 0, 0
        for _ in range(n):
            a = 0
            for j in range(nbits):
                if (f[cf] >> cb) & 1:
                    a |= 1 << j
                cb += 1
                if cb == 63:
                    cb, cf = 0, cf + 1
            res.append(a)
        return res


class GpuStarkKernels(GpuKernels):
    """libzkgpu device primitives on column-major torch tensors (ld = row
    count of the tensor unless given)."""

    def zeros(self, shape):
        return self.torch.zeros(shape, dtype=self.torch.int64, device=self.device)

    def rand_cols(self, t, ld, cols, nrows, seed, stream):
        cols = np.ascontiguousarray(cols, np.uint32)
        if cols.size:
            self.zk._check(self.zk.lib().zkgpu_rand_cols_dev(t.data_ptr(), ld, cols.ctypes.data, cols.size, nrows,
                                                             seed, stream), "zkgpu_rand_cols_dev")

    def zxp(self, prog, secs, log_dom, ch, pub, evals=None, xdiv=None, xdivw=None, eb=0, x_start=1):
        self.zk.zxp_eval_dev(prog, secs, log_dom, ch, pub, evals, xdiv, xdivw, extend_bits=eb, x_start=x_start)

    def zxp_block(self, prog, secs, log_rows, log_domain, ch, pub, evals, xdiv, xdivw, eb, x_start):
        self.zk.zxp_eval_block_dev(prog, secs, log_rows, log_domain, ch, pub, evals, xdiv, xdivw, extend_bits=eb,
                                   x_start=x_start)

    def h1h2(self, h1, h2, f, t, n, dim):
        return self.zk.h1h2_dev(h1, n, h2, n, f, n, t, n, n, dim)

    def calculate_z(self, z, num, den, n):
        return self.zk.calculate_z_dev(z, n, num, n, den, n, n)

    def ntt(self, dst, src, n, ncols, inverse=False):
        self.zk.ntt_dev(dst, dst.shape[-1], src, src.shape[-1], n, ncols, inverse)

    def qsplit(self, qq2, qq1, n, q_deg, shift_in):
        self.zk.qsplit_dev(qq2, qq2.shape[-1], qq1, qq1.shape[-1], n, q_deg, shift_in)

    def ext_powers(self, out, base, n):
        self.zk.ext_powers_dev(out, out.shape[-1], np.asarray(base, np.uint64), n)

    def evmap(self, cols, lds, dims, primes, lev, lpev, l_ld, n, eb):
        return self.zk.evmap_dev(cols, lds, dims, primes, lev, lpev, l_ld, n, eb)

    def xdivxsub(self, xdiv, xdivw, xi, n_bits, n_bits_ext):
        self.zk.xdivxsub_dev(xdiv, xdivw, np.asarray(xi, np.uint64), n_bits, n_bits_ext)

    def fri_fold(self, out, pol, pol_bits, out_bits, sx, shift_inv):
        self.zk.fri_fold_dev(out, pol, pol_bits, out_bits, np.asarray(sx, np.uint64), shift_inv)

    def fri_transpose(self, aux, pol, degree, bits):
        self.zk.fri_transpose_dev(aux, pol, degree, bits)

    def merkle_rows(self, src, ncols, nrows):
        nodes = self.empty(self.zk.merkle_num_elements(nrows))
        self.zk.merkletree_rows_dev(nodes, src, ncols, nrows)
        return nodes

    def open_rows(self, nodes, src, ncols, nrows, idx):
        return self.zk.merkle_open_rows_dev(nodes, src, ncols, nrows, np.asarray(idx, np.uint64))

    def hash_full(self, x):
        return self.zk.poseidon_full_host(x)

    def to_host(self, t):
        return self.zk.from_device(t.contiguous())


class ShardedStark:
    """genProof of one SyntheticStark instance, rows of the extended domain
    sharded over the process group (module docstring)."""

    def __init__(self, inst, group=None, kernels=None, device=None):
        import torch.distributed as dist
        self.inst, self.group = inst, group
        self.W = dist.get_world_size(group) if dist.is_initialized() else 1
        self.r = dist.get_rank(group) if dist.is_initialized() else 0
        self.k = kernels if kernels is not None else GpuStarkKernels(device)
        self.nb, self.nbe, self.eb = inst.n_bits, inst.n_bits_ext, inst.blowup_bits
        self.N, self.NE = 1 << self.nb, 1 << self.nbe
        if self.W & (self.W - 1) or self.NE % self.W:
            raise ValueError("world size must be a power of two dividing the extended domain")
        self.B = self.NE // self.W
        self.halo = 1 << self.eb  # row shift of next-row reads on the 2n domain
        if self.B < max(self.halo, 1 << self.eb):
            raise ValueError("row block smaller than the halo")
        k, N = self.k, self.N
        self.S = {0: k.zeros((max(inst.n_cm1, 1), N)), 1: k.zeros((max(inst.n_cm2, 1), N)),
                  2: k.zeros((max(inst.n_cm3, 1), N)), 3: k.zeros((max(inst.n_tmp, 1), N)),
                  4: k.zeros((inst.n_const, N))}
        self.timers = {}
        self._setup()

    # ------------------------------------------------------------ helpers
    def _secs_n(self):
        return {s: (t, self.N, t.shape[0]) for s, t in self.S.items()}

    def _commit(self, sec, ncols):
        c = ShardedCommit(self.nb, self.eb, ncols, self.group, kernels=self.k)
        root = c.commit(self.S[sec][c.lo:c.hi])
        return c, root

    def _with_halo(self, block):
        """ncols x B block -> ncols x (B + halo): the next block's first rows appended."""
        first = block[:, :self.halo].contiguous()
        nxt = all_gather(first, self.group)[(self.r + 1) % self.W]
        out = self.k.empty((block.shape[0], self.B + self.halo))
        out[:, :self.B] = block
        out[:, self.B:] = nxt
        return out

    def _gather_rows(self, t):
        """all-gather of ncols x B blocks -> ncols x NE (rank order)."""
        import torch
        return torch.cat(all_gather(t.contiguous(), self.group), dim=1)

    def _setup(self):
        inst, k, N = self.inst, self.k, self.N
        k.rand_cols(self.S[4], N, inst.random_const_cols(), N, inst.seed, 1)
        self.S[4][inst.l_first, 0] = 1
        from .synthetic import rand_u64
        self.publics = np.array([rand_u64(inst.seed, 2, j, 0) for j in range(inst.n_publics)], np.uint64)
        zero_ch = np.zeros((8, 3), np.uint64)
        if inst.programs["step0"].instr:
            k.zxp(inst.programs["step0"], self._secs_n(), self.nb, zero_ch, self.publics, eb=self.eb)
        self.const, self.verkey = self._commit(4, inst.n_const)
        self.const_h = self._with_halo(self.const.block)

    def witness(self):
        """Executor stand-in: pseudo-random cm1 columns + the step1 derivation."""
        inst, k = self.inst, self.k
        k.rand_cols(self.S[0], self.N, inst.random_cm1_cols(), self.N, inst.seed, 0)
        k.zxp(inst.programs["step1"], self._secs_n(), self.nb, np.zeros((8, 3), np.uint64), self.publics,
              eb=self.eb)

    # ------------------------------------------------------------ prove
    def prove_json(self):
        """The proof in the reference's zkin layout (canonical decimal strings)."""
        return to_json(self.prove())

    def prove(self):
        """The proof as arrays (roots, evals, openings, final polynomial)."""
        import time
        inst, k, S = self.inst, self.k, self.S
        N, NE, B, eb, nb, nbe = self.N, self.NE, self.B, self.eb, self.nb, self.nbe
        T = {}
        clock = [time.perf_counter()]

        def lap(name):
            k.synchronize()
            now = time.perf_counter()
            T[name] = (now - clock[0]) * 1e3
            clock[0] = now

        t = Transcript(k.hash_full)
        t.put(self.verkey)
        t.put(self.publics)
        ch = np.zeros((8, 3), np.uint64)
        # STAGE 1
        c1, root1 = self._commit(0, inst.n_cm1)
        t.put(root1)
        lap("STARK_STEP_1_COMMIT")
        # STAGE 2
        ch[0] = t.get_field()
        ch[1] = t.get_field()
        k.zxp(inst.programs["step2"], self._secs_n(), nb, ch, self.publics, eb=eb)
        for f_c, t_c, h1_c, h2_c, d in inst.pu:
            miss = k.h1h2(S[1][h1_c:h1_c + d], S[1][h2_c:h2_c + d], S[3][f_c:f_c + d], S[3][t_c:t_c + d], N, d)
            if miss is not None:
                raise ValueError("calculateH1H2: Number not included: w=%d" % miss)
        c2, root2 = self._commit(1, inst.n_cm2)
        t.put(root2)
        lap("STARK_STEP_2")
        # STAGE 3
        ch[2] = t.get_field()
        ch[3] = t.get_field()
        k.zxp(inst.programs["step3prev"], self._secs_n(), nb, ch, self.publics, eb=eb)
        for num_c, den_c, z_c in inst.z_ctx:
            if not k.calculate_z(S[2][z_c:z_c + 3], S[3][num_c:num_c + 3], S[3][den_c:den_c + 3], N):
                raise ValueError("calculateZ: the grand product does not close")
        if "step3" in inst.programs and inst.programs["step3"].instr:
            k.zxp(inst.programs["step3"], self._secs_n(), nb, ch, self.publics, eb=eb)  # starks.cpp:193
        c3, root3 = self._commit(2, inst.n_cm3)
        t.put(root3)
        lap("STARK_STEP_3")
        # STAGE 4: quotient on this rank's rows, then split + commit
        ch[4] = t.get_field()
        b1, b2, b3 = self._with_halo(c1.block), self._with_halo(c2.block), self._with_halo(c3.block)
        Bh = B + self.halo
        x0 = 7 * pow(w_of(nbe), self.r * B, P) % P
        log_b = B.bit_length() - 1
        q = k.zeros((3, B))
        secs = {5: (b1, Bh, inst.n_cm1), 6: (b2, Bh, max(inst.n_cm2, 1)), 7: (b3, Bh, max(inst.n_cm3, 1)),
                9: (self.const_h, Bh, inst.n_const), 10: (q, B, 3)}
        k.zxp_block(inst.programs["step42ns"], secs, log_b, nbe, ch, self.publics, None, None, None, eb, x0)
        qfull = self._gather_rows(q)
        qq1 = k.zeros((3, NE))
        k.ntt(qq1, qfull, NE, 3, inverse=True)
        qq2 = k.zeros((inst.q_deg * 3, NE))
        k.qsplit(qq2, qq1, N, inst.q_deg, pow(pow(7, P - 2, P), N, P))
        cm4 = k.zeros((inst.q_deg * 3, NE))
        k.ntt(cm4, qq2, NE, inst.q_deg * 3)
        c4 = ShardedCommit(nb, eb, inst.n_cm4, self.group, kernels=k)
        root4 = c4.commit_rows(cm4[:, self.r * B:(self.r + 1) * B].contiguous())
        del cm4, qq2, qq1, qfull
        t.put(root4)
        lap("STARK_STEP_4")
        # STAGE 5
        ch[7] = t.get_field()
        xi = [int(v) for v in ch[7]]
        inv7 = pow(7, P - 2, P)
        wN = w_of(nb)
        lev, lpev = k.zeros((3, N)), k.zeros((3, N))
        k.ext_powers(lev, [v * inv7 % P for v in xi], N)
        k.ext_powers(lpev, [v * wN % P * inv7 % P for v in xi], N)
        k.ntt(lev, lev, N, 3, inverse=True)
        k.ntt(lpev, lpev, N, 3, inverse=True)
        blocks = {5: (b1, Bh), 6: (b2, Bh), 7: (b3, Bh), 8: (c4.block, B), 9: (self.const_h, Bh)}
        k0, nloc = (self.r * B) >> eb, B >> eb
        cols = [blocks[sec][0][c] for sec, c, _, _ in inst.evmap]
        lds = np.array([blocks[sec][1] for sec, _, _, _ in inst.evmap], np.uint64)
        dims = [d for _, _, d, _ in inst.evmap]
        primes = [pr for _, _, _, pr in inst.evmap]
        part = k.evmap(cols, lds, dims, primes, lev[:, k0:], lpev[:, k0:], N, nloc, eb)
        import torch
        parts = all_gather(torch.from_numpy(np.ascontiguousarray(part).view(np.int64)), self.group)
        evals = np.zeros(part.shape, np.uint64)
        acc = np.zeros(part.shape, dtype=object)
        for p_ in parts:
            acc = acc + p_.cpu().numpy().view(np.uint64).astype(object)
        evals[:] = (acc % P).astype(np.uint64)
        t.put(evals)
        ch[5] = t.get_field()
        ch[6] = t.get_field()
        xdiv, xdivw = k.zeros(3 * NE), k.zeros(3 * NE)
        k.xdivxsub(xdiv, xdivw, ch[7], nb, nbe)
        f = k.zeros((3, B))
        secs = {5: (b1, Bh, inst.n_cm1), 6: (b2, Bh, max(inst.n_cm2, 1)), 7: (b3, Bh, max(inst.n_cm3, 1)),
                8: (c4.block, B, inst.n_cm4), 9: (self.const_h, Bh, inst.n_const), 11: (f, B, 3)}
        lo, hi = 3 * self.r * B, 3 * (self.r + 1) * B
        k.zxp_block(inst.programs["step52ns"], secs, log_b, nbe, ch, self.publics, evals, xdiv[lo:hi],
                    xdivw[lo:hi], eb, x0)
        pol = self._gather_rows(f).t().contiguous().reshape(-1)  # interleaved F_p^3 (NE x 3)
        del xdiv, xdivw, b1, b2, b3
        lap("STARK_STEP_5")
        out = self._fri(t, pol, [c1, c2, c3, c4, self.const], [root1, root2, root3, root4], evals)
        lap("STARK_STEP_FRI")
        T["STARK_TOTAL"] = sum(T.values())
        self.timers = T
        return out

    def _fri(self, t, pol, trees, roots, evals):
        """FRIProve::prove (friProve.cpp:5-190) on every rank, then queries."""
        inst, k = self.inst, self.k
        steps = inst.fri_steps
        pol_bits = self.nbe
        shift_inv = pow(7, P - 2, P)
        fri = [None]
        out = {}
        for si in range(len(steps)):
            red = pol_bits - steps[si]
            sx = t.get_field()
            if si > 0:
                nxt = k.zeros(3 << steps[si])
                k.fri_fold(nxt, pol, pol_bits, steps[si], sx, shift_inv)
                pol = nxt
            if si < len(steps) - 1:
                nbits = steps[si + 1]
                ngroups = 1 << nbits
                width = (3 << steps[si]) // ngroups
                aux = k.zeros(3 << steps[si])
                k.fri_transpose(aux, pol, 1 << steps[si], nbits)
                nodes = k.merkle_rows(aux, width, ngroups)
                fri.append((nodes, aux, width, ngroups))
                root = k.root(nodes)
                t.put(root)
                out["s%d_root" % (si + 1)] = root
            else:
                final = k.to_host(pol)
                t.put(final)
            pol_bits = steps[si]
            for _ in range(red):
                shift_inv = shift_inv * shift_inv % P
        out["finalPol"] = final.reshape(-1, 3)
        ys = t.get_permutations(inst.n_queries, steps[0])
        # s0: the rank owning a query row opens it in every stage tree
        per_tree = [c.open_local_many(ys) for c in trees]
        mine = [(qi, [op[y] for op in per_tree]) for qi, y in enumerate(ys) if y // self.B == self.r]
        import torch.distributed as dist
        if self.W > 1:
            got = [None] * self.W
            dist.all_gather_object(got, mine, group=self.group)
        else:
            got = [mine]
        opened = {}
        for lst in got:
            for qi, per_tree in lst:
                opened[qi] = per_tree
        tags = ["1", "2", "3", "4", "C"]
        for ti, tag in enumerate(tags):
            out["s0_vals" + tag] = np.array([opened[q][ti][0] for q in range(len(ys))], np.uint64)
            out["s0_siblings" + tag] = np.array([opened[q][ti][1] for q in range(len(ys))], np.uint64)
        # FRI layers (replicated trees)
        yq = list(ys)
        for si in range(1, len(steps)):
            yq = [y % (1 << steps[si]) for y in yq]
            nodes, aux, width, ngroups = fri[si]
            vals, sibs = k.open_rows(nodes, aux, width, ngroups, yq)
            out["s%d_vals" % si] = vals
            out["s%d_siblings" % si] = sibs
        out["root1"], out["root2"], out["root3"], out["root4"] = roots
        out["evals"] = evals
        return out
