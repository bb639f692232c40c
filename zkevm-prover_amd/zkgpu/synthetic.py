"""Synthetic starkinfo-shaped STARK instance.

The real fork-9 zkEVM instance cannot run here (its starkinfo, constant tree,
verkey and input are absent, and its memory map exceeds one GPU), so the
full-STARK workload is a synthetic AIR with the same stage structure as
Starks::genProof (starks.cpp:9-404):

  constants  K_0..K_{nK-1} (pseudo-random), L_first (1 at row 0)
  stage 1    cm1 = 3t columns; a[3j], a[3j+1] pseudo-random,
             a[3j+2] = a[3j]*a[3j+1]*K_{j mod nK} + a[3j]             (degree 3)
  lookups    n_lookups plookups (0..2) against constant tables:
             #0 dim 3: (A, B) in (T0, T1) combined as f = A + u B, t = T0 + u T1
             #1 dim 1: C in T2, T2 = T0 with row 0 replaced by T0[N/2] (a
                duplicate value, so the "last table row" rule matters)
             A, B, C are cm1 columns filled from the tables at shifted rows
  stage 2    challenges u = ch[0], defVal = ch[1];
             m extension columns h_j = sum_k a[s_j+k] u^(k+1) + defVal (cm2, 3m cols);
             plookup f/t into tmpExp, then h1/h2 = calculateH1H2(f, t) (cm2)
  stage 3    challenges gamma = ch[2], beta = ch[3];
             num_j = (h_j(x) + gamma) beta, den_j = (h_j(w x) + gamma) beta (tmpExp)
             Z_j = grand product of num_j/den_j (calculateZ, polinomial.hpp:586-607);
             it closes because den is num shifted by one row (cm3, 3m cols);
             plookup Z: num = (1+beta)(gamma+f)(gamma(1+beta) + t + beta t'),
             den = (gamma(1+beta) + h1 + beta h2)(gamma(1+beta) + h2 + beta h1')
  stage 4    alpha = ch[4]; C = Horner_alpha of all constraints; q = C / Z_H
             (step42ns semantics, op 69), split into qDeg = 2 pieces (cm4, 6 cols)
  stage 5    xi = ch[7]; evals (evmap); v1 = ch[5], v2 = ch[6];
             f = Horner_v1(committed cols) + Horner_v2(p - p(xi)) x/(x-xi)
                 + Horner_v2(p' - p(w xi)) x/(x - w xi)                (step52ns form)
  FRI        FRIProve::prove (friProve.cpp), queries on the 5 trees.

Width fillers (n_free2 / n_free_tmp / n_free3; the fork-9 widths 751 / 168 /
408 / 389 tmpExp / 234 constants, commit_pols.hpp:1736-1737):
extra committed / tmpExp columns derived row-locally by the stage programs --
step2: cm2 fillers from cm1 (one factor at the next row) and the constants;
step3prev: tmpExp fillers from the cm2 fillers at the next row; step3: cm3
fillers from the tmpExp fillers at the next row, every other one stored at
the next row (the shifted stores of step3.parser.cpp opcodes 101-114).  They
are committed, evaluated (evMap) and enter the FRI polynomial like every
committed column; no constraint reads them.

The constraint/expression programs are emitted in the ZXP format
(include/zkgpu_zxp.h) and evaluated by the GPU expression kernel (product) and
by the oracle's C evaluator (tests).  The instance is valid: a correct prover
produces a proof whose FRI layers are consistent and whose final polynomial
has degree < 2^last / blowup.
"""
import numpy as np

# kinds / ops / sections mirror include/zkgpu_zxp.h
TMP1, TMP3, COL, COL3, LIT, CHAL, PUB, X, EVAL, XDIV, XDIVW, ZI = range(12)
ADD, SUB, MUL, COPY = range(4)
(SEC_CM1_N, SEC_CM2_N, SEC_CM3_N, SEC_TMP_N, SEC_CONST_N, SEC_CM1_2NS, SEC_CM2_2NS, SEC_CM3_2NS, SEC_CM4_2NS,
 SEC_CONST_2NS, SEC_Q_2NS, SEC_F_2NS) = range(12)
SEC_N_TO_2NS = {SEC_CM1_N: SEC_CM1_2NS, SEC_CM2_N: SEC_CM2_2NS, SEC_CM3_N: SEC_CM3_2NS, SEC_CONST_N: SEC_CONST_2NS}

P = 0xFFFFFFFF00000001


class Program:
    """Builder for one ZXP program; operands are interned."""

    def __init__(self, domain_ext):
        self.domain_ext = int(domain_ext)
        self.opnd = []
        self._idx = {}
        self.instr = []
        self.n_tmp1 = 0
        self.n_tmp3 = 0

    def o(self, kind, a=0, b=0, c=0):
        key = (kind, a & 0xFFFFFFFF, b & 0xFFFFFFFF, c & 0xFFFFFFFF)
        if key not in self._idx:
            self._idx[key] = len(self.opnd)
            self.opnd.append(key)
        return self._idx[key]

    def tmp1(self):
        self.n_tmp1 += 1
        return self.o(TMP1, self.n_tmp1 - 1)

    def tmp3(self):
        self.n_tmp3 += 1
        return self.o(TMP3, self.n_tmp3 - 1)

    def col(self, sec, c, shift=0):
        return self.o(COL, sec, c, shift)

    def col3(self, sec, c, shift=0):
        return self.o(COL3, sec, c, shift)

    def lit(self, v):
        v %= P
        return self.o(LIT, v & 0xFFFFFFFF, v >> 32)

    def chal(self, k):
        return self.o(CHAL, k)

    def ev(self, k):
        return self.o(EVAL, k)

    def op(self, op, dst, a, b=0):
        self.instr.append((op, dst, a, b))
        return dst

    def arrays(self):
        ins = np.array(self.instr, dtype=np.uint32).reshape(-1, 4)
        opn = np.array(self.opnd, dtype=np.uint32).reshape(-1, 4)
        return ins, opn


class SyntheticStark:
    def __init__(self, n_bits=10, blowup_bits=1, t=4, m=2, n_k=3, n_queries=16, fri_steps=None, n_publics=8,
                 seed=0x5EED, n_free=0, n_lookups=2, q_deg=2, with_step3=True, n_free2=0, n_free3=0, n_free_tmp=0):
        self.n_bits = n_bits
        self.n_bits_ext = n_bits + blowup_bits
        self.blowup_bits = blowup_bits
        self.t, self.m, self.n_k = t, m, n_k
        self.n_free = n_free  # extra free (unconstrained, random) committed columns
        assert 0 <= n_lookups <= 2
        self.n_lookups = n_lookups
        # constants: K_0..K_{nK-1}, L_first, then the lookup tables
        self.l_first = n_k  # const column index of L_first
        self.c_t = [n_k + 1, n_k + 2, n_k + 3][:(2 if n_lookups >= 1 else 0) + (1 if n_lookups >= 2 else 0)]
        self.n_const = n_k + 1 + len(self.c_t)
        # cm1: 3t triples, n_free free columns, then lookup columns A, B, C
        base = 3 * t + n_free
        self.cm1_lk = list(range(base, base + len(self.c_t)))
        self.n_cm1 = base + len(self.c_t)
        # plookup contexts: dim, f/t tmp cols, h1/h2 cm2 cols, num/den tmp cols, Z cm3 col
        self.lookups = []
        cm2, tmp, cm3 = 3 * m, 6 * m, 3 * m
        for k in range(n_lookups):
            d = 3 if k == 0 else 1
            lk = {"dim": d, "f": tmp, "t": tmp + d, "h1": cm2, "h2": cm2 + d, "num": tmp + 2 * d,
                  "den": tmp + 2 * d + 3, "z": cm3}
            self.lookups.append(lk)
            cm2 += 2 * d
            tmp += 2 * d + 6
            cm3 += 3
        self.cm2_free = list(range(cm2, cm2 + n_free2))
        self.n_cm2 = cm2 + n_free2
        # post-Z stage-3 column (starks.cpp:193-208: step3 runs after calculateZ
        # and writes cm3/tmpExp columns that depend on Z): W = Z_0 * a_0 + K_0
        # (an F_p^3 column: the verifier only sees whole evaluations of Z)
        self.with_step3 = bool(with_step3)
        self.cm3_w = cm3 if self.with_step3 else None
        cm3 += 3 if self.with_step3 else 0
        self.cm3_free = list(range(cm3, cm3 + n_free3))
        self.n_cm3 = cm3 + n_free3
        self.tmp_free = list(range(tmp, tmp + n_free_tmp))
        self.n_tmp = tmp + n_free_tmp
        # quotient pieces: the constraints have degree <= 3, so pieces >= 2 are
        # zero polynomials; q_deg > 2 (blowup >= 4) still exercises the split
        assert 2 <= q_deg <= (1 << blowup_bits)
        self.q_deg, self.q_dim = q_deg, 3
        self.n_cm4 = self.q_deg * self.q_dim
        self.n_queries = n_queries
        self.n_publics = n_publics
        self.seed = seed
        if fri_steps is None:
            fri_steps = [self.n_bits_ext]
            while fri_steps[-1] - 4 >= max(5, blowup_bits + 3):
                fri_steps.append(fri_steps[-1] - 4)
        self.fri_steps = fri_steps
        # stage-2 groups: partition the cm1 columns into m contiguous groups
        cols = list(range(self.n_cm1))
        size = (len(cols) + m - 1) // m
        self.groups = [cols[j * size:(j + 1) * size] for j in range(m)]
        assert all(self.groups), "too many stage-2 groups for the cm1 width"
        self.z_ctx = [(6 * j, 6 * j + 3, 3 * j) for j in range(m)]  # (num tmp col, den tmp col, z cm3 col)
        self.z_ctx += [(lk["num"], lk["den"], lk["z"]) for lk in self.lookups]
        self.pu = [(lk["f"], lk["t"], lk["h1"], lk["h2"], lk["dim"]) for lk in self.lookups]
        self._build_evmap()
        self.programs = {
            "step0": self._prog_step0(),
            "step1": self._prog_step1(),
            "step2": self._prog_step2(),
            "step3prev": self._prog_step3prev(),
            "step3": self._prog_step3(),
            "step42ns": self._prog_step42ns(),
            "step52ns": self._prog_step52ns(),
        }

    # ------------------------------------------------------------ evMap
    def _build_evmap(self):
        """evMap entries (section_2ns, col, dim, prime), in the order the
        transcript absorbs the evals (starks.cpp:336-339)."""
        ev = []
        for c in range(self.n_cm1):
            ev.append((SEC_CM1_2NS, c, 1, 0))
        for k in range(self.n_const):
            ev.append((SEC_CONST_2NS, k, 1, 0))
        for c in self.c_t:
            ev.append((SEC_CONST_2NS, c, 1, 1))  # t' in the plookup Z
        for j in range(self.m):
            ev.append((SEC_CM2_2NS, 3 * j, 3, 0))
            ev.append((SEC_CM2_2NS, 3 * j, 3, 1))
        for lk in self.lookups:
            ev.append((SEC_CM2_2NS, lk["h1"], lk["dim"], 0))
            ev.append((SEC_CM2_2NS, lk["h1"], lk["dim"], 1))
            ev.append((SEC_CM2_2NS, lk["h2"], lk["dim"], 0))
        for j in range(self.m):
            ev.append((SEC_CM3_2NS, 3 * j, 3, 0))
            ev.append((SEC_CM3_2NS, 3 * j, 3, 1))
        for lk in self.lookups:
            ev.append((SEC_CM3_2NS, lk["z"], 3, 0))
            ev.append((SEC_CM3_2NS, lk["z"], 3, 1))
        if self.with_step3:
            ev.append((SEC_CM3_2NS, self.cm3_w, 3, 0))
        for j, c in enumerate(self.cm2_free):
            ev.append((SEC_CM2_2NS, c, 1, 0))
            if j % 4 == 0:
                ev.append((SEC_CM2_2NS, c, 1, 1))
        for c in self.cm3_free:
            ev.append((SEC_CM3_2NS, c, 1, 0))
        for p in range(self.q_deg):
            ev.append((SEC_CM4_2NS, 3 * p, 3, 0))
        self.evmap = ev
        self.ev_index = {(s, c, pr): i for i, (s, c, d, pr) in enumerate(ev)}

    # ------------------------------------------------------------ programs
    def _prog_step0(self):
        """Constant derivation (setup): T2 = T0 with row 0 := T0[N/2]."""
        p = Program(0)
        if len(self.c_t) < 3:
            return p
        t = p.tmp1()
        t0, lf = p.col(SEC_CONST_N, self.c_t[0]), p.col(SEC_CONST_N, self.l_first)
        p.op(SUB, t, p.col(SEC_CONST_N, self.c_t[0], 1 << (self.n_bits - 1)), t0)
        p.op(MUL, t, t, lf)
        p.op(ADD, t, t, t0)
        p.op(COPY, p.col(SEC_CONST_N, self.c_t[2]), t)
        return p

    # rows of the tables the lookup columns read: A, B at T[i+5] (row 0: T[11]), C at T2[i+7]
    LK_SHIFT, LK_SHIFT0, LK_SHIFT_C = 5, 11, 7

    def _prog_step1(self):
        """Trace derivation (executor stand-in): a[3j+2] = a[3j] a[3j+1] K_j + a[3j];
        lookup columns copied from table rows."""
        p = Program(0)
        t = p.tmp1()
        for j in range(self.t):
            a0, a1, a2 = (p.col(SEC_CM1_N, 3 * j + k) for k in range(3))
            kk = p.col(SEC_CONST_N, j % self.n_k)
            p.op(MUL, t, a0, a1)
            p.op(MUL, t, t, kk)
            p.op(ADD, t, t, a0)
            p.op(COPY, a2, t)
        lf = p.col(SEC_CONST_N, self.l_first)
        for k, c in enumerate(self.cm1_lk[:2]):
            tc = self.c_t[k]
            p.op(SUB, t, p.col(SEC_CONST_N, tc, self.LK_SHIFT0), p.col(SEC_CONST_N, tc, self.LK_SHIFT))
            p.op(MUL, t, t, lf)
            p.op(ADD, t, t, p.col(SEC_CONST_N, tc, self.LK_SHIFT))
            p.op(COPY, p.col(SEC_CM1_N, c), t)
        if len(self.cm1_lk) > 2:
            p.op(COPY, p.col(SEC_CM1_N, self.cm1_lk[2]), p.col(SEC_CONST_N, self.c_t[2], self.LK_SHIFT_C))
        return p

    def _lk_ft(self, p, k, cm1_sec, const_sec, shift_t):
        """(f, t') operands/temps of plookup k: f = A + u B | C, t = T0 + u T1 | T2 (row shift shift_t)."""
        if self.lookups[k]["dim"] == 3:
            u = p.chal(0)
            f = p.tmp3()
            p.op(MUL, f, u, p.col(cm1_sec, self.cm1_lk[1]))
            p.op(ADD, f, f, p.col(cm1_sec, self.cm1_lk[0]))
            t = p.tmp3()
            p.op(MUL, t, u, p.col(const_sec, self.c_t[1], shift_t))
            p.op(ADD, t, t, p.col(const_sec, self.c_t[0], shift_t))
            return f, t
        return p.col(cm1_sec, self.cm1_lk[2]), p.col(const_sec, self.c_t[2], shift_t)

    def _lk_col(self, p, sec, c, dim, shift=0):
        return p.col3(sec, c, shift) if dim == 3 else p.col(sec, c, shift)

    def _emit_lk_num_den(self, p, lk, f, t, t_next, h1, h2, h1_next, num, den):
        """num = (1+beta)(gamma+f)(gamma(1+beta) + t + beta t'),
        den = (gamma(1+beta) + h1 + beta h2)(gamma(1+beta) + h2 + beta h1')."""
        gamma, beta = p.chal(2), p.chal(3)
        ob = p.tmp3()
        p.op(ADD, ob, beta, p.lit(1))
        gb = p.tmp3()
        p.op(MUL, gb, ob, gamma)
        x = p.tmp3()
        y = p.tmp3()
        p.op(ADD, x, f, gamma)
        p.op(MUL, x, x, ob)
        p.op(MUL, y, beta, t_next)
        p.op(ADD, y, y, t)
        p.op(ADD, y, y, gb)
        p.op(MUL, num, x, y)
        p.op(MUL, x, beta, h2)
        p.op(ADD, x, x, h1)
        p.op(ADD, x, x, gb)
        p.op(MUL, y, beta, h1_next)
        p.op(ADD, y, y, h2)
        p.op(ADD, y, y, gb)
        p.op(MUL, den, x, y)
        return num, den

    def _emit_h(self, p, grp, sec, shift, dst3):
        """dst3 = sum_k a[s+k] u^(k+1) + defVal over the group's columns."""
        u = p.chal(0)
        dv = p.chal(1)
        cols = grp
        p.op(MUL, dst3, u, p.col(sec, cols[-1], shift))
        for c in reversed(cols[:-1]):
            p.op(ADD, dst3, dst3, p.col(sec, c, shift))
            p.op(MUL, dst3, dst3, u)
        p.op(ADD, dst3, dst3, dv)
        return dst3

    def _prog_step2(self):
        p = Program(0)
        h = p.tmp3()
        for j, grp in enumerate(self.groups):
            self._emit_h(p, grp, SEC_CM1_N, 0, h)
            p.op(COPY, p.col3(SEC_CM2_N, 3 * j), h)
        # plookup f / t into tmpExp (transposeH1H2Columns reads them, starks.cpp:406-438)
        for k, lk in enumerate(self.lookups):
            f, t = self._lk_ft(p, k, SEC_CM1_N, SEC_CONST_N, 0)
            p.op(COPY, self._lk_col(p, SEC_TMP_N, lk["f"], lk["dim"]), f)
            p.op(COPY, self._lk_col(p, SEC_TMP_N, lk["t"], lk["dim"]), t)
        # cm2 fillers: a * b' + K
        if self.cm2_free:
            r = p.tmp1()
            for j, c in enumerate(self.cm2_free):
                p.op(MUL, r, p.col(SEC_CM1_N, (7 * j) % self.n_cm1), p.col(SEC_CM1_N, (13 * j + 5) % self.n_cm1, 1))
                p.op(ADD, p.col(SEC_CM2_N, c), r, p.col(SEC_CONST_N, j % self.n_const))
        return p

    def _prog_step3prev(self):
        p = Program(0)
        t = p.tmp3()
        gamma, beta = p.chal(2), p.chal(3)
        for j in range(self.m):
            num_c, den_c, _ = self.z_ctx[j]
            p.op(ADD, t, p.col3(SEC_CM2_N, 3 * j, 0), gamma)
            p.op(MUL, p.col3(SEC_TMP_N, num_c), t, beta)
            p.op(ADD, t, p.col3(SEC_CM2_N, 3 * j, 1), gamma)
            p.op(MUL, p.col3(SEC_TMP_N, den_c), t, beta)
        for lk in self.lookups:
            d = lk["dim"]
            f = self._lk_col(p, SEC_TMP_N, lk["f"], d)
            tt = self._lk_col(p, SEC_TMP_N, lk["t"], d)
            tn = self._lk_col(p, SEC_TMP_N, lk["t"], d, 1)
            h1 = self._lk_col(p, SEC_CM2_N, lk["h1"], d)
            h2 = self._lk_col(p, SEC_CM2_N, lk["h2"], d)
            h1n = self._lk_col(p, SEC_CM2_N, lk["h1"], d, 1)
            self._emit_lk_num_den(p, lk, f, tt, tn, h1, h2, h1n, p.col3(SEC_TMP_N, lk["num"]),
                                  p.col3(SEC_TMP_N, lk["den"]))
        # tmpExp fillers: (cm2 filler)' + a
        for j, c in enumerate(self.tmp_free):
            src = (p.col(SEC_CM2_N, self.cm2_free[j % len(self.cm2_free)], 1) if self.cm2_free
                   else p.col(SEC_CM1_N, j % self.n_cm1, 1))
            p.op(ADD, p.col(SEC_TMP_N, c), src, p.col(SEC_CM1_N, (11 * j) % self.n_cm1))
        return p

    def _prog_step3(self):
        """Post-Z stage-3 expressions (starks.cpp:193): W = Z_0 * a_0 + K_0."""
        p = Program(0)
        if not self.with_step3:
            return p
        t = p.tmp3()
        z0 = self.z_ctx[0][2]
        p.op(MUL, t, p.col3(SEC_CM3_N, z0), p.col(SEC_CM1_N, 0))
        p.op(ADD, p.col3(SEC_CM3_N, self.cm3_w), t, p.col(SEC_CONST_N, 0))
        # cm3 fillers: (tmpExp filler)' * a + K, odd ones stored at the next row
        if self.cm3_free:
            r = p.tmp1()
            for j, c in enumerate(self.cm3_free):
                src = (p.col(SEC_TMP_N, self.tmp_free[j % len(self.tmp_free)], 1) if self.tmp_free
                       else p.col(SEC_CM1_N, j % self.n_cm1, 1))
                p.op(MUL, r, src, p.col(SEC_CM1_N, (17 * j + 1) % self.n_cm1))
                p.op(ADD, p.col(SEC_CM3_N, c, j % 2), r, p.col(SEC_CONST_N, (3 * j) % self.n_const))
        return p

    def constraints(self, p, nxt):
        """Yield (emit_fn) for each constraint; each writes its value into a
        fresh temp and returns it.  nxt = row shift of "next row"."""
        out = []
        for j in range(self.t):
            def c_mul(j=j):
                r = p.tmp1()
                a0, a1, a2 = (p.col(SEC_CM1_2NS, 3 * j + k) for k in range(3))
                p.op(MUL, r, a0, a1)
                p.op(MUL, r, r, p.col(SEC_CONST_2NS, j % self.n_k))
                p.op(ADD, r, r, a0)
                p.op(SUB, r, a2, r)
                return r
            out.append(c_mul)
        for j, grp in enumerate(self.groups):
            def c_h(j=j, grp=grp):
                r = p.tmp3()
                self._emit_h(p, grp, SEC_CM1_2NS, 0, r)
                p.op(SUB, r, p.col3(SEC_CM2_2NS, 3 * j), r)
                return r
            out.append(c_h)
        for j in range(self.m):
            def c_first(j=j):
                r = p.tmp3()
                p.op(SUB, r, p.col3(SEC_CM3_2NS, 3 * j), p.lit(1))
                p.op(MUL, r, r, p.col(SEC_CONST_2NS, self.l_first))
                return r
            out.append(c_first)
        for j in range(self.m):
            def c_z(j=j):
                gamma, beta = p.chal(2), p.chal(3)
                r = p.tmp3()
                s = p.tmp3()
                p.op(ADD, r, p.col3(SEC_CM2_2NS, 3 * j, nxt), gamma)
                p.op(MUL, r, r, beta)
                p.op(MUL, r, r, p.col3(SEC_CM3_2NS, 3 * j, nxt))
                p.op(ADD, s, p.col3(SEC_CM2_2NS, 3 * j, 0), gamma)
                p.op(MUL, s, s, beta)
                p.op(MUL, s, s, p.col3(SEC_CM3_2NS, 3 * j, 0))
                p.op(SUB, r, r, s)
                return r
            out.append(c_z)
        if self.with_step3:
            def c_w():
                r = p.tmp3()
                p.op(MUL, r, p.col3(SEC_CM3_2NS, self.z_ctx[0][2]), p.col(SEC_CM1_2NS, 0))
                p.op(ADD, r, r, p.col(SEC_CONST_2NS, 0))
                p.op(SUB, r, p.col3(SEC_CM3_2NS, self.cm3_w), r)
                return r
            out.append(c_w)
        for k, lk in enumerate(self.lookups):
            def c_lk_first(lk=lk):
                r = p.tmp3()
                p.op(SUB, r, p.col3(SEC_CM3_2NS, lk["z"]), p.lit(1))
                p.op(MUL, r, r, p.col(SEC_CONST_2NS, self.l_first))
                return r

            def c_lk_z(k=k, lk=lk):
                d = lk["dim"]
                f, t = self._lk_ft(p, k, SEC_CM1_2NS, SEC_CONST_2NS, 0)
                _, tn = self._lk_ft(p, k, SEC_CM1_2NS, SEC_CONST_2NS, nxt)
                h1 = self._lk_col(p, SEC_CM2_2NS, lk["h1"], d)
                h2 = self._lk_col(p, SEC_CM2_2NS, lk["h2"], d)
                h1n = self._lk_col(p, SEC_CM2_2NS, lk["h1"], d, nxt)
                num, den = self._emit_lk_num_den(p, lk, f, t, tn, h1, h2, h1n, p.tmp3(), p.tmp3())
                r = p.tmp3()
                p.op(MUL, r, den, p.col3(SEC_CM3_2NS, lk["z"], nxt))
                p.op(MUL, num, num, p.col3(SEC_CM3_2NS, lk["z"]))
                p.op(SUB, r, r, num)
                return r
            out.append(c_lk_first)
            out.append(c_lk_z)
        return out

    def _prog_step42ns(self):
        p = Program(1)
        nxt = 1 << self.blowup_bits
        alpha = p.chal(4)
        acc = p.tmp3()
        first = True
        for emit in self.constraints(p, nxt):
            r = emit()
            if first:
                p.op(COPY, acc, r)
                first = False
            else:
                p.op(MUL, acc, acc, alpha)
                p.op(ADD, acc, acc, r)
        p.op(MUL, p.col3(SEC_Q_2NS, 0), acc, p.o(ZI))
        return p

    def committed_columns(self):
        """(section, col, dim) of every committed polynomial, Horner order of f."""
        cols = [(SEC_CM1_2NS, c, 1) for c in range(self.n_cm1)]
        cols += [(SEC_CM2_2NS, 3 * j, 3) for j in range(self.m)]
        for lk in self.lookups:
            cols += [(SEC_CM2_2NS, lk["h1"], lk["dim"]), (SEC_CM2_2NS, lk["h2"], lk["dim"])]
        cols += [(SEC_CM3_2NS, 3 * j, 3) for j in range(self.m)]
        cols += [(SEC_CM3_2NS, lk["z"], 3) for lk in self.lookups]
        if self.with_step3:
            cols += [(SEC_CM3_2NS, self.cm3_w, 3)]
        cols += [(SEC_CM2_2NS, c, 1) for c in self.cm2_free]
        cols += [(SEC_CM3_2NS, c, 1) for c in self.cm3_free]
        cols += [(SEC_CM4_2NS, 3 * q, 3) for q in range(self.q_deg)]
        return cols

    def _prog_step52ns(self):
        p = Program(1)
        v1, v2 = p.chal(5), p.chal(6)
        acc = p.tmp3()
        first = True
        for sec, c, dim in self.committed_columns():
            opnd = p.col(sec, c) if dim == 1 else p.col3(sec, c)
            if first:
                p.op(MUL, acc, opnd, v1)  # promote to F_p^3 via v1 (reference op 0: T0 = pols * v1)
                first = False
            else:
                p.op(MUL, acc, acc, v1)
                p.op(ADD, acc, acc, opnd)
        for prime, xdiv in ((0, XDIV), (1, XDIVW)):
            g = p.tmp3()
            d = p.tmp3()
            firstg = True
            for i, (sec, c, dim, pr) in enumerate(self.evmap):
                if pr != prime:
                    continue
                opnd = p.col(sec, c) if dim == 1 else p.col3(sec, c)
                p.op(SUB, d, opnd, p.ev(i))
                if firstg:
                    p.op(COPY, g, d)
                    firstg = False
                else:
                    p.op(MUL, g, g, v2)
                    p.op(ADD, g, g, d)
            p.op(MUL, g, g, p.o(xdiv))
            p.op(ADD, acc, acc, g)
        p.op(COPY, p.col3(SEC_F_2NS, 0), acc)
        return p

    # ------------------------------------------------------------ description
    def info(self):
        return {
            "nBits": self.n_bits, "nBitsExt": self.n_bits_ext, "nQueries": self.n_queries,
            "friSteps": self.fri_steps, "nCm1": self.n_cm1, "nCm2": self.n_cm2, "nCm3": self.n_cm3,
            "nCm4": self.n_cm4, "nTmp": self.n_tmp, "nConst": self.n_const, "nPublics": self.n_publics,
            "qDeg": self.q_deg, "qDim": self.q_dim, "lFirst": self.l_first, "seed": self.seed,
            "randomCm1Cols": self.random_cm1_cols(), "randomConst": self.random_const_cols(),
            "zCtx": self.z_ctx, "puCtx": self.pu, "evMap": self.evmap,
        }

    @classmethod
    def fork9(cls, n_bits=10, **kw):
        """The fork-9 zkEVM widths (commit_pols.hpp:1736-1737):
        cm1 / cm2 / cm3 / cm4 = 751 / 168 / 408 / 6 committed columns, 234
        constants, 389 tmpExp columns, two plookups, blowup 2."""
        a = dict(n_bits=n_bits, blowup_bits=1, t=4, m=2, n_k=230, n_free=736, n_lookups=2, q_deg=2,
                 n_free2=154, n_free3=393, n_free_tmp=357, n_queries=8)
        a.update(kw)
        inst = cls(**a)
        assert (inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4, inst.n_const, inst.n_tmp) == \
            (751, 168, 408, 6, 234, 389), "fork-9 widths"
        return inst

    def random_cm1_cols(self):
        return [c for c in range(3 * self.t + self.n_free) if c >= 3 * self.t or c % 3 != 2]

    def random_const_cols(self):
        """K_k and the random tables T0, T1 (T2 is derived by step0)."""
        return list(range(self.n_k)) + self.c_t[:2]


# ---------------------------------------------------------------- PRNG
MASK64 = (1 << 64) - 1


def rand_u64(seed, stream, col, row):
    """Deterministic pseudo-random canonical element (splitmix64 finaliser);
    the same function is implemented by the GPU trace generator
    (csrc/stark.hip k_rand_cols) and the oracle (oracle/stark.c)."""
    x = (seed ^ (stream << 56) ^ (col * 0x9E3779B97F4A7C15) ^ (row * 0xC2B2AE3D27D4EB4F)) & MASK64
    z = (x + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    z ^= z >> 31
    return z >> 1
