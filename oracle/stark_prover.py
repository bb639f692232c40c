"""oracle/stark_prover.py -- TEST INFRASTRUCTURE ONLY.

CPU restatement of Starks::genProof (starks.cpp:9-404) and FRIProve::prove
(friProve.cpp:5-190) for a SyntheticStark instance, orchestrated in Python
over the C oracle (row-major sections, like the reference's memory map).
Produces the proof in the reference's zkin layout (proof2zkinStark.cpp:8-82)
with canonical decimal strings.  Used by tests/ and bench.py's cpu_baseline.
"""
import ctypes

import numpy as np

from . import oracle as oc

P = 0xFFFFFFFF00000001


def _p(a):
    return oc._p(a)


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data)


class OracleStark:
    def __init__(self, inst):
        self.inst = inst
        self.N = 1 << inst.n_bits
        self.NE = 1 << inst.n_bits_ext
        self.eb = inst.blowup_bits
        L = oc.lib()
        N, NE = self.N, self.NE
        S = {}
        S[0] = np.zeros((N, max(inst.n_cm1, 1)), np.uint64)
        S[1] = np.zeros((N, max(inst.n_cm2, 1)), np.uint64)
        S[2] = np.zeros((N, max(inst.n_cm3, 1)), np.uint64)
        S[3] = np.zeros((N, max(inst.n_tmp, 1)), np.uint64)
        S[4] = np.zeros((N, inst.n_const), np.uint64)
        self.S = S
        # constants (setup, like the reference's const pols + const tree files)
        kcols = np.array(inst.random_const_cols(), dtype=np.uint32)
        L.oc_rand_cols(_p(S[4]), inst.n_const, _vp(kcols), kcols.size, N, inst.seed, 1)
        S[4][0, inst.l_first] = 1
        self.publics = np.array([L.oc_rand_u64(inst.seed, 2, k, 0) for k in range(inst.n_publics)], np.uint64)
        self.x_n = np.zeros(N, np.uint64)
        L.oc_powers(_p(self.x_n), 1, oc.gl_w(inst.n_bits), N)
        self.x_2ns = np.zeros(NE, np.uint64)
        L.oc_powers(_p(self.x_2ns), 7, oc.gl_w(inst.n_bits_ext), NE)
        # zhInv (zhInv.cpp:7-31)
        sn = pow(7, N, P)
        wE = oc.gl_w(self.eb)
        self.zhinv = np.array([pow((sn * pow(wE, i, P) - 1) % P, P - 2, P) for i in range(1 << self.eb)], np.uint64)
        # derived constants (step0), then the constant LDE + tree -> verkey
        if inst.programs["step0"].instr:
            self.run(inst.programs["step0"], np.zeros(3 * 8, np.uint64), np.zeros(3, np.uint64))
        S[9] = oc.extend_pol(S[4], NE)
        self.const_nodes = oc.merkletree(S[9])
        self.verkey = self.const_nodes[-4:].copy()

    # ------------------------------------------------------------ helpers
    def witness(self):
        """cm1_n: pseudo-random columns + the step1 derivation (executor stand-in)."""
        inst = self.inst
        rc = np.array(inst.random_cm1_cols(), dtype=np.uint32)
        oc.lib().oc_rand_cols(_p(self.S[0]), self.S[0].shape[1], _vp(rc), rc.size, self.N, inst.seed, 0)
        self.run(inst.programs["step1"], np.zeros(3 * 8, np.uint64), np.zeros(3, np.uint64))

    def run(self, prog, challenges, evals, xdiv=None, xdivw=None):
        ins, opn = prog.arrays()
        dom = self.NE if prog.domain_ext else self.N
        secs = (ctypes.c_void_p * 12)()
        strides = np.zeros(12, np.uint64)
        keep = []
        for k, a in self.S.items():
            secs[k] = a.ctypes.data
            strides[k] = a.shape[1]
        x = self.x_2ns if prog.domain_ext else self.x_n
        xd = xdiv if xdiv is not None else np.zeros(3, np.uint64)
        xw = xdivw if xdivw is not None else np.zeros(3, np.uint64)
        keep.append((ins, opn))
        oc.lib().oc_zxp_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                             max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ctypes.cast(secs, ctypes.c_void_p),
                             ctypes.c_void_p(strides.ctypes.data), dom, _p(np.ascontiguousarray(challenges)),
                             _p(self.publics), _p(np.ascontiguousarray(evals)), _p(x), _p(xd), _p(xw),
                             _p(self.zhinv), self.zhinv.size)

    # ------------------------------------------------------------ prove
    def prove(self):
        inst = self.inst
        N, NE, S = self.N, self.NE, self.S
        t = oc.Transcript()
        t.put(self.verkey)
        t.put(self.publics)
        ch = np.zeros((8, 3), np.uint64)
        roots = []
        trees = []
        # STAGE 1 (starks.cpp:49-63)
        S[5] = oc.extend_pol(S[0], NE)
        trees.append((oc.merkletree(S[5]), S[5]))
        roots.append(trees[-1][0][-4:].copy())
        t.put(roots[-1])
        # STAGE 2 (:65-144)
        ch[0] = t.get_field()
        ch[1] = t.get_field()
        self.run(inst.programs["step2"], ch, np.zeros(3, np.uint64))
        # plookups: h1/h2 = calculateH1H2(f, t) (starks.cpp:104-127)
        for f_c, t_c, h1_c, h2_c, d in inst.pu:
            fcol = np.ascontiguousarray(S[3][:, f_c:f_c + d])
            tcol = np.ascontiguousarray(S[3][:, t_c:t_c + d])
            h1, h2 = oc.h1h2(fcol.reshape(-1) if d == 1 else fcol, tcol.reshape(-1) if d == 1 else tcol)
            S[1][:, h1_c:h1_c + d] = h1.reshape(N, d)
            S[1][:, h2_c:h2_c + d] = h2.reshape(N, d)
        S[6] = oc.extend_pol(S[1], NE)
        trees.append((oc.merkletree(S[6]), S[6]))
        roots.append(trees[-1][0][-4:].copy())
        t.put(roots[-1])
        # STAGE 3 (:146-224)
        ch[2] = t.get_field()
        ch[3] = t.get_field()
        self.run(inst.programs["step3prev"], ch, np.zeros(3, np.uint64))
        for num_c, den_c, z_c in inst.z_ctx:
            zc = np.zeros((N, 3), np.uint64)
            num = np.ascontiguousarray(S[3][:, num_c:num_c + 3])
            den = np.ascontiguousarray(S[3][:, den_c:den_c + 3])
            ok = oc.lib().oc_calculate_z(_p(zc), 3, _p(num), 3, _p(den), 3, N)
            assert ok, "calculateZ: product does not close"
            S[2][:, z_c:z_c + 3] = zc
        # step3: post-Z expressions (starks.cpp:193-208)
        if "step3" in inst.programs and inst.programs["step3"].instr:
            self.run(inst.programs["step3"], ch, np.zeros(3, np.uint64))
        S[7] = oc.extend_pol(S[2], NE)
        trees.append((oc.merkletree(S[7]), S[7]))
        roots.append(trees[-1][0][-4:].copy())
        t.put(roots[-1])
        # STAGE 4 (:226-296)
        ch[4] = t.get_field()
        S[10] = np.zeros((NE, 3), np.uint64)
        self.run(inst.programs["step42ns"], ch, np.zeros(3, np.uint64))
        qq1 = oc.ntt(S[10], True)
        shift_in = pow(pow(7, P - 2, P), N, P)
        qq2 = np.zeros((NE, inst.q_deg * 3), np.uint64)
        cur = 1
        for p in range(inst.q_deg):
            blk = qq1[p * N:(p + 1) * N]
            qq2[:N, 3 * p:3 * p + 3] = (blk.astype(object) * cur % P).astype(np.uint64)
            cur = cur * shift_in % P
        S[8] = oc.ntt(qq2)
        trees.append((oc.merkletree(S[8]), S[8]))
        roots.append(trees[-1][0][-4:].copy())
        t.put(roots[-1])
        # STAGE 5 (:298-392)
        ch[7] = t.get_field()
        xi = [int(v) for v in ch[7]]
        inv7 = pow(7, P - 2, P)
        xis = np.array([v * inv7 % P for v in xi], np.uint64)
        wN = oc.gl_w(inst.n_bits)
        wxis = np.array([v * wN % P * inv7 % P for v in xi], np.uint64)
        lev = self._powers3(xis, N)
        lpev = self._powers3(wxis, N)
        lev = oc.ntt(lev, True)
        lpev = oc.ntt(lpev, True)
        evals = self.evmap(lev, lpev)
        t.put(evals)
        ch[5] = t.get_field()
        ch[6] = t.get_field()
        xdiv = np.zeros((NE, 3), np.uint64)
        xdivw = np.zeros((NE, 3), np.uint64)
        oc.lib().oc_xdivxsub(_p(xdiv), _p(xdivw), _p(self.x_2ns), NE, _p(ch[7].copy()), wN)
        S[11] = np.zeros((NE, 3), np.uint64)
        self.run(inst.programs["step52ns"], ch, evals, xdiv, xdivw)
        self.challenges = ch
        self.evals = evals
        return self._fri(t, trees, roots, evals)

    def _powers3(self, base, n):
        out = np.zeros((n, 3), np.uint64)
        oc.lib().oc_powers3(_p(out), _p(np.ascontiguousarray(base, dtype=np.uint64)), n)
        return out

    def evmap(self, lev, lpev):
        inst = self.inst
        n_ev = len(inst.evmap)
        ptrs = (ctypes.c_void_p * n_ev)()
        strides = np.zeros(n_ev, np.uint64)
        dims = np.zeros(n_ev, np.uint32)
        primes = np.zeros(n_ev, np.uint32)
        for e, (sec, c, dim, pr) in enumerate(inst.evmap):
            a = self.S[sec]
            ptrs[e] = a.ctypes.data + 8 * c
            strides[e] = a.shape[1]
            dims[e] = dim
            primes[e] = pr
        evals = np.zeros((n_ev, 3), np.uint64)
        oc.lib().oc_evmap(_p(evals), ctypes.cast(ptrs, ctypes.c_void_p), ctypes.c_void_p(strides.ctypes.data),
                          ctypes.c_void_p(dims.ctypes.data), ctypes.c_void_p(primes.ctypes.data), n_ev,
                          _p(np.ascontiguousarray(lev)), _p(np.ascontiguousarray(lpev)), self.N, self.eb)
        return evals

    def _fri(self, t, trees, roots, evals):
        """FRIProve::prove (friProve.cpp:5-190) + queries, zkin layout."""
        inst = self.inst
        steps = inst.fri_steps
        pol = np.ascontiguousarray(self.S[11]).reshape(-1)
        pol_bits = inst.n_bits_ext
        shift_inv = pow(7, P - 2, P)
        fri_trees = [None]
        fri_srcs = [None]
        proof = {}
        for si in range(len(steps)):
            red = pol_bits - steps[si]
            sx = t.get_field()
            if si == 0:
                pol2 = pol.copy()
            else:
                pol2 = oc.fri_fold(pol, pol_bits, steps[si], sx, shift_inv)
            if si < len(steps) - 1:
                nb = steps[si + 1]
                aux = oc.fri_get_transposed(pol2, nb)
                ngroups = 1 << nb
                src = aux.reshape(ngroups, -1)
                nodes = oc.merkletree(src)
                fri_trees.append(nodes)
                fri_srcs.append(src)
                t.put(nodes[-4:])
                proof["s%d_root" % (si + 1)] = nodes[-4:].copy()
            else:
                t.put(pol2)
            pol = pol2
            pol_bits = steps[si]
            for _ in range(red):
                shift_inv = shift_inv * shift_inv % P
        final = pol.reshape(-1, 3)
        ys = [int(y) for y in t.get_permutations(inst.n_queries, steps[0])]
        # queries (friProve.cpp:156-178)
        all_trees = [(n, s) for n, s in trees] + [(self.const_nodes, self.S[9])]
        tags = ["1", "2", "3", "4", "C"]
        for tag in tags:
            proof["s0_vals" + tag] = []
            proof["s0_siblings" + tag] = []
        for si in range(1, len(steps)):
            proof["s%d_vals" % si] = []
            proof["s%d_siblings" % si] = []
        for si in range(len(steps)):
            for q in range(inst.n_queries):
                if si == 0:
                    for tag, (nodes, src) in zip(tags, all_trees):
                        v, s = oc.merkle_group_proof(nodes, src, ys[q])
                        proof["s0_vals" + tag].append(v)
                        proof["s0_siblings" + tag].append(s)
                else:
                    v, s = oc.merkle_group_proof(fri_trees[si], fri_srcs[si], ys[q])
                    proof["s%d_vals" % si].append(v)
                    proof["s%d_siblings" % si].append(s)
            if si < len(steps) - 1:
                ys = [y % (1 << steps[si + 1]) for y in ys]
        proof["root1"], proof["root2"], proof["root3"], proof["root4"] = roots
        proof["evals"] = evals
        proof["finalPol"] = final
        return to_json(proof)


def to_json(proof):
    """canonical decimal strings, zkin layout"""
    def conv(v):
        if isinstance(v, np.ndarray):
            return conv(v.tolist())
        if isinstance(v, list):
            return [conv(x) for x in v]
        return str(int(v) % P)
    order = ["root1", "root2", "root3", "root4", "evals"]
    out = {k: conv(proof[k]) for k in order}
    i = 1
    while "s%d_root" % i in proof:
        for k in ("root", "vals", "siblings"):
            out["s%d_%s" % (i, k)] = conv(proof["s%d_%s" % (i, k)])
        i += 1
    for tag in ("1", "2", "3", "4", "C"):
        out["s0_vals" + tag] = conv(proof["s0_vals" + tag])
    for tag in ("1", "2", "3", "4", "C"):
        out["s0_siblings" + tag] = conv(proof["s0_siblings" + tag])
    out["finalPol"] = conv(proof["finalPol"])
    return out
