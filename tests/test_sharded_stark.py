"""Row-sharded full STARK (zkgpu/sharded_stark.py) vs the single-process proof.

CPU (gloo, world sizes 1, 2, 4): the whole distributed prover -- sharded
commits, halos, row-block quotient and FRI programs, the q / f gathers,
evmap partial sums, owner-served openings -- with oracle-backed CPU kernels
(test infrastructure) injected; the proof must equal the oracle prover's
(oracle/stark_prover.py) byte for byte.
GPU: world 1 on the HIP kernels, and world 2 as two processes sharing the one
GPU (collectives staged through the host over gloo) -- the same proof.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_sharded import OracleKernels

P = 0xFFFFFFFF00000001


def _u(t):
    return t.numpy().view(np.uint64)


class OracleStarkKernels(OracleKernels):
    """CPU stand-ins for GpuStarkKernels (column-major int64 torch tensors)."""

    def zeros(self, shape):
        return torch.zeros(shape, dtype=torch.int64)

    def rand_cols(self, t, ld, cols, nrows, seed, stream):
        for c in cols:
            col = np.array([self.oc.lib().oc_rand_u64(seed, stream, int(c), r) for r in range(nrows)], np.uint64)
            t[int(c), :nrows] = torch.from_numpy(col.view(np.int64))

    def _run(self, prog, secs, dom, x, ch, pub, evals, xdiv, xdivw, zh):
        """oc_zxp_eval on row-major copies (dom rows each), results copied back."""
        L = self.oc.lib()
        rm = {}
        sp = (ctypes.c_void_p * 12)()
        strides = np.zeros(12, np.uint64)
        for s, (t, ld, nc) in secs.items():
            a = np.zeros((dom, max(nc, 1)), np.uint64)
            rows = min(dom, t.shape[1])
            a[:rows, :t.shape[0]] = _u(t)[:, :rows].T
            rm[s] = a
            sp[s] = a.ctypes.data
            strides[s] = a.shape[1]
        ins, opn = prog.arrays()
        ins, opn = np.ascontiguousarray(ins), np.ascontiguousarray(opn)
        p = self.oc._p
        ch = np.ascontiguousarray(ch, np.uint64).reshape(-1)
        pub = np.ascontiguousarray(pub if pub is not None and len(pub) else np.zeros(1), np.uint64)
        ev = np.ascontiguousarray(evals if evals is not None else np.zeros(3), np.uint64).reshape(-1)
        xd = np.ascontiguousarray(xdiv if xdiv is not None else np.zeros(3), np.uint64).reshape(-1)
        xw = np.ascontiguousarray(xdivw if xdivw is not None else np.zeros(3), np.uint64).reshape(-1)
        L.oc_zxp_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                      max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ctypes.cast(sp, ctypes.c_void_p),
                      ctypes.c_void_p(strides.ctypes.data), dom, p(ch), p(pub), p(ev), p(x), p(xd), p(xw), p(zh),
                      zh.size)
        return rm

    def _zh(self, log_omega, eb):
        n = 1 << (log_omega - eb)
        we = self.oc.gl_w(eb)
        return np.array([pow((pow(7, n, P) * pow(we, i, P) - 1) % P, P - 2, P) for i in range(1 << eb)], np.uint64)

    def zxp(self, prog, secs, log_dom, ch, pub, evals=None, xdiv=None, xdivw=None, eb=0, x_start=1):
        dom = 1 << log_dom
        w = self.oc.gl_w(log_dom)
        x = np.array([x_start * pow(w, i, P) % P for i in range(dom)], np.uint64)
        rm = self._run(prog, secs, dom, x, ch, pub, evals, xdiv, xdivw, self._zh(log_dom, eb))
        for s, (t, ld, nc) in secs.items():
            t[:, :dom] = torch.from_numpy(np.ascontiguousarray(rm[s][:, :t.shape[0]].T).view(np.int64))

    def zxp_block(self, prog, secs, log_rows, log_domain, ch, pub, evals, xdiv, xdivw, eb, x_start):
        rows = 1 << log_rows
        dom = max(t.shape[1] for t, _, _ in secs.values())  # block + halo; rows >= B are discarded
        w = self.oc.gl_w(log_domain)
        x = np.array([x_start * pow(w, i, P) % P for i in range(dom)], np.uint64)

        def pad(a):
            if a is None:
                return None
            a = _u(a).reshape(-1, 3)
            out = np.zeros((dom, 3), np.uint64)
            out[:a.shape[0]] = a
            return out
        rm = self._run(prog, secs, dom, x, ch, pub, evals, pad(xdiv), pad(xdivw), self._zh(log_domain, eb))
        for s, (t, ld, nc) in secs.items():
            n = min(rows, t.shape[1])
            t[:, :n] = torch.from_numpy(np.ascontiguousarray(rm[s][:n, :t.shape[0]].T).view(np.int64))

    def h1h2(self, h1, h2, f, t, n, dim):
        fv, tv = _u(f)[:, :n].T, _u(t)[:, :n].T
        try:
            a, b = self.oc.h1h2(fv.reshape(-1) if dim == 1 else fv, tv.reshape(-1) if dim == 1 else tv)
        except ValueError:
            return 0
        h1[:, :n] = torch.from_numpy(np.ascontiguousarray(a.reshape(n, dim).T).view(np.int64))
        h2[:, :n] = torch.from_numpy(np.ascontiguousarray(b.reshape(n, dim).T).view(np.int64))
        return None

    def calculate_z(self, z, num, den, n):
        zc = np.zeros((n, 3), np.uint64)
        nm = np.ascontiguousarray(_u(num)[:, :n].T)
        dn = np.ascontiguousarray(_u(den)[:, :n].T)
        p = self.oc._p
        ok = self.oc.lib().oc_calculate_z(p(zc), 3, p(nm), 3, p(dn), 3, n)
        z[:, :n] = torch.from_numpy(np.ascontiguousarray(zc.T).view(np.int64))
        return bool(ok)

    def ntt(self, dst, src, n, ncols, inverse=False):
        r = self.oc.ntt(np.ascontiguousarray(_u(src)[:ncols, :n].T), inverse)
        dst[:ncols, :n] = torch.from_numpy(np.ascontiguousarray(r.T).view(np.int64))

    def qsplit(self, qq2, qq1, n, q_deg, shift_in):
        a = _u(qq1)
        f = 1
        for p_ in range(q_deg):
            for d in range(3):
                v = (a[d, p_ * n:(p_ + 1) * n].astype(object) * f % P).astype(np.uint64)
                qq2[3 * p_ + d, :n] = torch.from_numpy(v.view(np.int64))
            f = f * shift_in % P

    def ext_powers(self, out, base, n):
        cur = np.array([1, 0, 0], np.uint64)
        b = np.asarray(base, np.uint64)
        vals = np.zeros((n, 3), np.uint64)
        for k in range(n):
            vals[k] = cur
            cur = self.oc.gl3_mul(cur, b)
        out[:, :n] = torch.from_numpy(np.ascontiguousarray(vals.T).view(np.int64))

    def evmap(self, cols, lds, dims, primes, lev, lpev, l_ld, n, eb):
        n_ev = len(cols)
        keep = []
        ptrs = (ctypes.c_void_p * n_ev)()
        strides = np.zeros(n_ev, np.uint64)
        for e, (c, d) in enumerate(zip(cols, dims)):
            ld = int(lds[e])
            base = c.numpy().view(np.uint64)  # a view starting at the entry's first column
            flat = np.lib.stride_tricks.as_strided(base, shape=(d, ld), strides=(ld * 8, 8))
            rm = np.ascontiguousarray(flat.T)  # rows x d
            keep.append(rm)
            ptrs[e] = rm.ctypes.data
            strides[e] = d
        lv = np.ascontiguousarray(_u(lev)[:, :n].T)
        lp = np.ascontiguousarray(_u(lpev)[:, :n].T)
        out = np.zeros((n_ev, 3), np.uint64)
        p = self.oc._p
        dims_a = np.ascontiguousarray(dims, np.uint32)
        pr_a = np.ascontiguousarray(primes, np.uint32)
        self.oc.lib().oc_evmap(p(out), ctypes.cast(ptrs, ctypes.c_void_p), ctypes.c_void_p(strides.ctypes.data),
                               ctypes.c_void_p(dims_a.ctypes.data), ctypes.c_void_p(pr_a.ctypes.data), n_ev, p(lv),
                               p(lp), n, eb)
        return out

    def xdivxsub(self, xdiv, xdivw, xi, n_bits, n_bits_ext):
        ne = 1 << n_bits_ext
        w = self.oc.gl_w(n_bits_ext)
        x = np.array([7 * pow(w, i, P) % P for i in range(ne)], np.uint64)
        a, b = np.zeros((ne, 3), np.uint64), np.zeros((ne, 3), np.uint64)
        p = self.oc._p
        self.oc.lib().oc_xdivxsub(p(a), p(b), p(x), ne, p(np.ascontiguousarray(xi, np.uint64)),
                                  self.oc.gl_w(n_bits))
        xdiv[:] = torch.from_numpy(a.reshape(-1).view(np.int64))
        xdivw[:] = torch.from_numpy(b.reshape(-1).view(np.int64))

    def fri_fold(self, out, pol, pol_bits, out_bits, sx, shift_inv):
        r = self.oc.fri_fold(_u(pol), pol_bits, out_bits, np.asarray(sx, np.uint64), shift_inv)
        out[:] = torch.from_numpy(r.view(np.int64))

    def fri_transpose(self, aux, pol, degree, bits):
        aux[:] = torch.from_numpy(self.oc.fri_get_transposed(_u(pol), bits).view(np.int64))

    def merkle_rows(self, src, ncols, nrows):
        return torch.from_numpy(self.oc.merkletree(_u(src).reshape(nrows, ncols)).view(np.int64))

    def open_rows(self, nodes, src, ncols, nrows, idx):
        rows = _u(src).reshape(nrows, ncols)
        vs, ss = [], []
        for i in idx:
            v, s = self.oc.merkle_group_proof(_u(nodes), rows, int(i))
            vs.append(v)
            ss.append(s)
        return np.array(vs), np.array(ss)

    def hash_full(self, x):
        return self.oc.poseidon_full(x)

    def to_host(self, t):
        return _u(t).copy()


def _instance():
    from zkgpu.synthetic import SyntheticStark
    return SyntheticStark(n_bits=7, blowup_bits=1, t=3, m=2, n_free=2, n_lookups=2, n_queries=8)


def _oracle_proof(inst):
    from oracle.stark_prover import OracleStark
    o = OracleStark(inst)
    o.witness()
    return o.prove()


def _worker(rank, world, port, q, gpu):
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root_dir, os.path.join(root_dir, "zkevm-prover_amd"), os.path.join(root_dir, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from zkgpu.sharded_stark import ShardedStark
        if gpu:
            import zkgpu
            zkgpu.init(0)
            zkgpu.set_stream(torch.cuda.current_stream())
            s = ShardedStark(_instance(), device="cuda:0")
        else:
            from oracle import oracle as oc
            s = ShardedStark(_instance(), kernels=OracleStarkKernels(oc))
        s.witness()
        proof = s.prove_json()
        q.put((rank, proof, None))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_world(world, gpu=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, gpu)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [e for _, _, e in res if e]
    assert not errs, errs[0]
    return [pr for _, pr, _ in sorted(res, key=lambda x: x[0])]


@pytest.fixture(scope="module")
def reference_proof():
    return _oracle_proof(_instance())


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_stark_gloo_equals_single_process(reference_proof, world):
    proofs = _run_world(world)
    for pr in proofs:
        for k in reference_proof:
            assert pr[k] == reference_proof[k], k


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2])
def test_sharded_stark_gpu_equals_single_process(reference_proof, world):
    """HIP kernels; world 2 = two processes on the one GPU (host-staged gloo)."""
    proofs = _run_world(world, gpu=True)
    for pr in proofs:
        for k in reference_proof:
            assert pr[k] == reference_proof[k], k
