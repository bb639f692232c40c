"""The zkEVM-shaped STARK instance: the fork-9 widths with the five
zkEVM-shaped expression programs in the prover's stage slots.

Starks::genProof runs five bytecode programs (starks.cpp:73, 155, 193, 241,
371): step2prev / step3prev / step3 on the n domain, step42ns (the constraint
quotient, 18.5 K ops) and step52ns (the FRI polynomial over 1,973
evaluations) on the extended one.  The reference's programs and their
starkinfo are absent, so this instance takes
  * the fork-9 section widths (SyntheticStark.fork9: cm1 / cm2 / cm3 / cm4 =
    751 / 168 / 408 / 6, 389 tmpExp columns, 234 constants, two plookups,
    blowup 2) with its plookup (h1 / h2), grand-product (Z) and post-Z
    columns, which calculateH1H2 / calculateZ need to succeed;
  * the synthetic programs with the reference programs' shape
    (zkgpu/synthetic_bytecode.py: opcode histograms, temporaries, column
    reads and stores, row shifts, challenges, publics, evaluations), run
    through the product converter (zkgpu_parser_convert) exactly like the
    reference's bytecode:
      step2prev, step3prev, step3  appended to the instance's own stage
          programs; their stores go to the columns the instance does not own
          (the width fillers of cm2 / cm3 / tmpExp), their reads only to
          columns an earlier stage defined (or their own forwarded cells), so
          no kernel reads a cell another row of the same kernel writes;
      step42ns, step52ns  replace the instance's quotient and FRI polynomial.
  * an evaluation map of 1,973 entries (1,242 unprimed + 731 primed, the
    zkEVM's).
The quotient is not that of constraints the trace satisfies, so the proof
does not verify; every stage is still deterministic, and the GPU proof is
compared bit for bit with the oracle's (tests/test_gpu_zkevm_shaped.py).
"""
import numpy as np

from . import synthetic as sy
from . import synthetic_bytecode as sb

N_EV_ZKEVM = 1973          # evMap entries of the fork-9 zkEVM (step52ns bytecode)
N_EV_PRIMED_ZKEVM = 731
STAGE_PARSER = {"step2": "step2prev", "step3prev": "step3prev", "step3": "step3"}
SEC_NAME = {sy.SEC_CM1_N: "cm1_n", sy.SEC_CM2_N: "cm2_n", sy.SEC_CM3_N: "cm3_n", sy.SEC_TMP_N: "tmpExp_n"}
NAME_SEC = {v: k for k, v in SEC_NAME.items()}


def merge(a, b):
    """ZXP program a followed by b (operands re-interned, b's temporaries
    after a's)."""
    p = sy.Program(a.domain_ext)
    ia, oa = a.arrays()
    ib, ob = b.arrays()
    for prog, ins, opn, t1, t3 in ((a, ia, oa, 0, 0), (b, ib, ob, a.n_tmp1, a.n_tmp3)):
        idx = []
        for kind, x, y, z in opn.tolist():
            if kind == sy.TMP1:
                x += t1
            elif kind == sy.TMP3:
                x += t3
            idx.append(p.o(kind, x, y, z))
        for op, d, x, y in ins.tolist():
            p.op(op, idx[d], idx[x], idx[y])
    p.n_tmp1 = a.n_tmp1 + b.n_tmp1
    p.n_tmp3 = a.n_tmp3 + b.n_tmp3
    return p


def col_access(prog):
    """(reads, writes): sets of (section, column, row shift) of a ZXP program"""
    ins, opn = prog.arrays()
    opn = opn.tolist()
    writes = set()
    dsts = set()
    for op, d, x, y in ins.tolist():
        dsts.add(d)
        kind, s, c, sh = opn[d]
        if kind in (sy.COL, sy.COL3):
            for j in range(3 if kind == sy.COL3 else 1):
                writes.add((s, c + j, sh))
    reads = set()
    for op, d, x, y in ins.tolist():
        for o in ((x, y) if op != sy.COPY else (x,)):
            kind, s, c, sh = opn[o]
            if kind in (sy.COL, sy.COL3):
                for j in range(3 if kind == sy.COL3 else 1):
                    reads.add((s, c + j, sh))
    return reads, writes


class ZkevmShapedStark(sy.SyntheticStark):
    """SyntheticStark.fork9 with the zkEVM-shaped programs (module doc)."""

    def __init__(self, *a, program_seed=1, **kw):
        self.program_seed = program_seed
        super().__init__(*a, **kw)
        self.programs.update(self._build_programs())
        self.programs["step42ns"] = self._shaped("step42ns", None, None)
        self.programs["step52ns"] = self._shaped("step52ns", None, None)

    @classmethod
    def create(cls, n_bits=10, n_queries=8, fri_steps=None, program_seed=1):
        return cls.fork9(n_bits=n_bits, n_queries=n_queries, fri_steps=fri_steps, n_publics=48,
                         program_seed=program_seed)

    # ------------------------------------------------------------ evMap
    def _build_evmap(self):
        super()._build_evmap()
        ev = list(self.evmap)
        n_primed = sum(1 for e in ev if e[3])
        # unprimed cm1 entries are all present; add primed cm1 / cm3 / cm2
        # entries, then unprimed constants of the zkEVM's width, up to 1,973
        extra = [(sy.SEC_CM1_2NS, c, 1, 1) for c in range(self.n_cm1)]
        extra += [(sy.SEC_CM3_2NS, c, 1, 1) for c in self.cm3_free]
        have = {(s, c, pr) for s, c, d, pr in ev}
        for e in extra:
            if len(ev) >= N_EV_ZKEVM or n_primed >= N_EV_PRIMED_ZKEVM:
                break
            if (e[0], e[1], e[3]) not in have:
                ev.append(e)
                have.add((e[0], e[1], e[3]))
                n_primed += 1
        for c in self.cm3_free:
            if len(ev) >= N_EV_ZKEVM:
                break
            if (sy.SEC_CM3_2NS, c, 0) not in have:
                ev.append((sy.SEC_CM3_2NS, c, 1, 0))
                have.add((sy.SEC_CM3_2NS, c, 0))
        assert len(ev) == N_EV_ZKEVM, len(ev)
        self.evmap = ev
        self.ev_index = {(s, c, pr): i for i, (s, c, d, pr) in enumerate(ev)}

    # ------------------------------------------------------------ programs
    def _owned(self):
        """columns the instance's own logic writes (never written by the
        shaped programs): cm2 below its fillers (h groups, h1 / h2) and the
        fillers too (the instance's step2 writes them: cm2 is read whole by
        step3prev), cm3 below its fillers (Z, W), tmpExp below its fillers
        (plookup f / t, grand-product num / den)"""
        return {"cm2_n": set(range(self.n_cm2)),
                "cm3_n": set(range(self.cm3_free[0] if self.cm3_free else self.n_cm3)),
                "tmpExp_n": set(range(self.tmp_free[0] if self.tmp_free else self.n_tmp))}

    def _shaped(self, parser, reserved, readable):
        import zkgpu.parser as zp
        shape = sb.load_shape()
        ops, args = sb.generate(parser, seed=self.program_seed, shape=shape, reserved=reserved, readable=readable)
        return zp.convert(sb.PARSERS.index(parser), ops, args, sb.sections(shape), shape["n_bits"],
                          shape["n_bits_ext"])

    def _stage_programs(self):
        own = self._owned()
        lk_ft = set()
        for lk in self.lookups:
            lk_ft |= set(range(lk["f"], lk["f"] + lk["dim"])) | set(range(lk["t"], lk["t"] + lk["dim"]))
        z_cols = set()
        for _, _, z in self.z_ctx:
            z_cols |= {z, z + 1, z + 2}
        num_den = set()
        for num, den, _ in self.z_ctx:
            num_den |= {num, num + 1, num + 2, den, den + 1, den + 2}
        defined = {"cm3_n": set(), "tmpExp_n": set()}  # filler columns the shaped programs have written so far
        progs = {}
        # stage 2: step2prev reads cm1 (and its own stores)
        readable = {"cm2_n": set(), "cm3_n": set(), "tmpExp_n": set()}
        for slot, extra_cm3, extra_tmp in (("step2", set(), set()), ("step3prev", set(), lk_ft),
                                           ("step3", z_cols, lk_ft | num_den)):
            parser = STAGE_PARSER[slot]
            if slot != "step2":
                readable = {"cm2_n": set(range(self.n_cm2)), "cm3_n": defined["cm3_n"] | extra_cm3,
                            "tmpExp_n": defined["tmpExp_n"] | extra_tmp}
            prog = self._shaped(parser, own, readable)
            _, w = col_access(prog)
            for s, c, _ in w:
                assert SEC_NAME[s] in defined and c not in own[SEC_NAME[s]], (slot, s, c)
                defined[SEC_NAME[s]].add(c)
            progs[slot] = prog
        return progs

    def _build_programs(self):
        base_fill = (self.cm3_free, self.tmp_free)
        # the instance's own stage programs without the cm3 / tmpExp fillers
        # (those columns are the shaped programs'); cm2 fillers stay
        self.tmp_free, self.cm3_free = [], []
        own2, own3p, own3 = self._prog_step2(), self._prog_step3prev(), self._prog_step3()
        self.cm3_free, self.tmp_free = base_fill
        shaped = self._stage_programs()
        return {"step2": merge(own2, shaped["step2"]), "step3prev": merge(own3p, shaped["step3prev"]),
                "step3": merge(own3, shaped["step3"])}

