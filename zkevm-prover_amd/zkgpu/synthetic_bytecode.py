"""Synthetic Steps bytecode with the SHAPE of the reference's fork-9 programs.

The zkEVM bytecode (zkevm.chelpers.<step>.parser.hpp) cannot travel to the
GPU box and is not stored in the repository.  Its statistics can: op / arg
counts, temporaries, opcode histogram, the sections and columns it reads,
row shifts, challenge use (tests/golden/zkevm_bytecode_shape.json, written by
tools/bytecode_shape.py).  generate() builds a valid program in the same
instruction set (csrc/parser_isa.inc) with that histogram over the same
fork-9 memory map:

  * body: the non-chain opcodes in random order, operands drawn like the
    reference's (columns of the map's sections in proportion to its reads,
    next-row accesses at the program's row shift, constants, literals,
    challenges 0-3, publics);
  * results: a fraction of the base-field values are constraint results,
    folded into an F_p^3 accumulator by the fused Horner opcodes (step42ns
    84 / 87: acc = (acc + c) * challenges[4]) -- interleaved with the body so
    up to ~1,100 results are pending at once, as in the reference;
  * the final store (opcode 69, q_2ns = zhInv * acc).

The programs run through the product converter exactly like the reference's
and are checked against the oracle's case-table interpreter
(tests/test_gpu_parser.py) and timed at 2^24 rows (bench.py --workload step42ns).
"""
import json
import os
import re

import numpy as np

P = 0xFFFFFFFF00000001
HERE = os.path.dirname(os.path.abspath(__file__))
ISA_INC = os.path.join(os.path.dirname(HERE), "csrc", "parser_isa.inc")
SHAPE = os.path.join(os.path.dirname(os.path.dirname(HERE)), "tests", "golden", "zkevm_bytecode_shape.json")
PARSERS = ["step2prev", "step3prev", "step3", "step42ns", "step52ns"]
KINDS = {1: "T1", 2: "T3", 3: "P", 4: "PS", 5: "K", 6: "KS", 7: "KL", 8: "L", 9: "C", 10: "CL", 11: "U", 12: "E",
         13: "EL", 14: "X", 15: "ZI", 16: "XDIV", 17: "XDIVW", 18: "Q", 19: "F", 20: "A"}
OPS = {0: "add", 1: "sub", 2: "mul", 3: "copy", 4: "qout"}


def load_isa(path=ISA_INC):
    """{parser: {opcode: (nargs, [(op, dst, a, b)])}}, operand = (kind, dim, f0..f3)"""
    isa = {p: {} for p in PARSERS}
    num = r"(-?\d+)"
    opnd = r"\{%s, %s, \{%s, %s, %s, %s\}\}" % ((num,) * 6)
    row = re.compile(r"^\{%s, %s, %s, %s, %s, %s, %s\},$" % (num, num, num, num, opnd, opnd, opnd))
    for line in open(path):
        m = row.match(line.strip())
        if not m:
            continue
        g = [int(x) for x in m.groups()]
        pid, code, nargs, op = g[:4]
        ops = [tuple(g[4 + 6 * j:10 + 6 * j]) for j in range(3)]
        ent = isa[PARSERS[pid]].setdefault(code, (nargs, []))
        ent[1].append((OPS[op],) + tuple((KINDS.get(o[0]), o[1]) + tuple(o[2:]) if o[0] else None for o in ops))
    return isa


def load_shape(path=SHAPE):
    with open(path) as f:
        return json.load(f)


class _Gen:
    def __init__(self, name, shape, rng):
        self.name = name
        self.doc = shape
        self.sh = shape["programs"][name]
        self.rng = rng
        self.ext = name in ("step42ns", "step52ns")
        self.dom = 1 << (shape["n_bits_ext"] if self.ext else shape["n_bits"])
        self.row_shift = int(max(self.sh["row_shifts"], key=lambda k: self.sh["row_shifts"][k])) \
            if self.sh["row_shifts"] else (2 if self.ext else 1)
        self.map = {m["section"]: m for m in shape["map"]}
        reads = self.sh["reads"]
        self.rsecs = sorted(reads)
        w = np.array([reads[s]["accesses"] for s in self.rsecs], float)
        self.rprob = w / w.sum()
        # a fixed random column subset per section, the size of the reference's distinct set
        self.rcols = {}
        for s in self.rsecs:
            width = self.map[s]["width"]
            n = min(reads[s]["distinct_cols"], width)
            self.rcols[s] = np.sort(rng.choice(width, size=n, replace=False))
        self.n_const = shape["n_const"]
        self.chal = [int(c) for c in self.sh["challenges"] if int(c) != 4] or [0]
        self.n1 = max(self.sh["ntemp1"], 8)
        self.n3 = max(self.sh["ntemp3"], 4)

    def col(self, dim):
        s = self.rsecs[self.rng.choice(len(self.rsecs), p=self.rprob)]
        width = self.map[s]["width"]
        cols = self.rcols[s]
        c = int(cols[self.rng.integers(len(cols))])
        c = min(c, width - dim)
        return self.map[s]["offset"] + c, width


def generate(name="step42ns", seed=1, shape=None, isa=None, scale=1.0):
    """(ops, args) uint64 arrays of a synthetic program shaped like the
    reference's `name` program (currently step42ns: constraint quotient);
    scale < 1 keeps that fraction of every opcode count (same mix, same map).

    Values form constraint trees: an opcode's temporary operands are taken
    from the not-yet-used values (most recent first), its result joins them;
    the oldest unused values become constraint results once more than
    FRONTIER are waiting, and results are folded into the accumulator by the
    Horner opcodes.  No value is dead, as in the reference."""
    if name != "step42ns":
        raise NotImplementedError("synthetic shapes: step42ns")
    FRONTIER = 24
    shape = shape or load_shape()
    isa = isa or load_isa()
    table = isa[name]
    rng = np.random.default_rng(seed)
    g = _Gen(name, shape, rng)
    hist = {int(k): max(1, int(round(v * scale))) for k, v in g.sh["opcode_hist"].items()}
    n84, n87 = hist.pop(84, 0), hist.pop(87, 0)
    hist.pop(69, None)
    body = np.repeat(np.array(list(hist), np.int64), list(hist.values()))
    rng.shuffle(body)
    ops, args = [], []
    # T1 slots: free / unused values (frontier) / pending results;
    # T3 slot 0 = accumulator, 1 = chain scratch, 2.. values
    free1 = list(range(g.n1))
    free3 = list(range(2, g.n3))
    front1, front3, pending = [], [], []
    any1, any3 = [], []
    written1 = []  # T1 slots written at least once

    shared = []  # values used across many constraints (the reference's selectors / shared subexpressions)
    N_SHARED = 80

    def take(front, anyv):
        if anyv is any1 and len(shared) == N_SHARED and rng.random() < 0.08:
            return shared[int(rng.integers(N_SHARED))]
        if front and rng.random() < 0.9:
            return front.pop(len(front) - 1 - min(int(rng.exponential(2)), len(front) - 1))
        if anyv:
            return anyv[len(anyv) - 1 - min(int(rng.exponential(16)), len(anyv) - 1)]
        return None

    def chain(k):
        """k results (1 -> op 84, 4 -> op 87): acc = (acc + c) * alpha"""
        ops.append(84 if k == 1 else 87)
        for _ in range(k):
            c = pending.pop(0)
            args.extend([1, c, 0, 0, 4, 1])  # add13(t3[1] = t1[c] + t3[0]); mul33c(t3[0] = t3[1] * ch[4])
            free1.append(c)

    ops.append(13)  # acc = 0 + challenges[4] (add1c3c)
    args.extend([0, 0, 4])
    # a few column copies (opcode 79) first, so that every temporary an
    # opcode reads has been written before in the same row: the reference's
    # interpreters keep temporaries across rows, an unwritten one would carry
    # the previous row's value
    for _ in range(4):
        s_ = free1.pop(0)
        off, w = g.col(1)
        ops.append(79)
        args.extend([s_, off, w])
        written1.append(s_)
        front1.append(s_)
        any1.append(s_)
    for code in body:
        nargs, mops = table[int(code)]
        while len(free1) < 8:  # more open values than slots: fold some (past the quota if need be)
            if len(pending) < 4:
                pending.extend(front1[:4])
                del front1[:4]
            chain(4 if len(pending) >= 4 else 1)
        a = [0] * nargs
        filled = [False] * nargs
        released1, released3 = [], []

        def put(f, v):
            if f >= 0 and not filled[f]:
                a[f] = int(v)
                filled[f] = True
                return True
            return False

        for (op, d, x, y) in mops:
            for o in (x, y):  # operands first (defined values)
                if o is None:
                    continue
                k = o[0]
                if k == "T1" and not filled[o[2]]:
                    s_ = take(front1, any1)
                    if s_ is None:  # nothing open: any value written before
                        s_ = written1[int(rng.integers(len(written1)))]
                    released1.append(s_)
                    put(o[2], s_)
                elif k == "T3" and not filled[o[2]]:
                    s_ = take(front3, any3)
                    put(o[2], 0 if s_ is None else s_)
                    if s_ is not None:
                        released3.append(s_)
                elif k in ("P", "PS"):
                    off, w = g.col(o[1])
                    put(o[2], off)
                    if k == "P":
                        put(o[3], w)
                    else:
                        put(o[3], g.row_shift)
                        put(o[4], g.dom)
                        put(o[5], w)
                elif k == "K":
                    put(o[2], rng.integers(g.n_const))
                elif k == "KS":
                    put(o[2], rng.integers(g.n_const))
                    put(o[3], g.row_shift)
                    put(o[4], g.dom)
                elif k == "L":
                    put(o[2], int(rng.integers(0, P, dtype=np.uint64)) if rng.random() < 0.3
                        else int(rng.integers(0, 64)))
                elif k == "C":
                    put(o[2], g.chal[rng.integers(len(g.chal))])
                elif k == "U":
                    put(o[2], rng.integers(max(1, (g.sh["max_public"] or 0) + 1)))
            kd = d[0]
            if kd == "T1":
                s_ = free1.pop(0) if free1 else released1.pop()
                put(d[2], s_)
                if s_ not in written1:
                    written1.append(s_)
                if len(shared) < N_SHARED:
                    shared.append(s_)  # reserved for the whole program
                    if s_ in released1:
                        released1.remove(s_)
                else:
                    front1.append(s_)
                    any1.append(s_)
            elif kd == "T3":
                s_ = free3.pop(0) if free3 else (released3.pop() if released3 else 2 + int(rng.integers(g.n3 - 2)))
                put(d[2], s_)
                front3.append(s_)
                any3.append(s_)
        assert all(filled), (code, mops, filled)
        # operand slots whose values are no longer waiting become free
        for s_ in released1:
            if s_ not in front1 and s_ not in pending and s_ not in free1 and s_ not in shared:
                free1.append(s_)
        for s_ in released3:
            if s_ not in front3 and s_ not in free3:
                free3.append(s_)
        any1[:] = any1[-256:]
        any3[:] = any3[-64:]
        ops.append(int(code))
        args.extend(a)
        while len(front1) > FRONTIER:
            pending.append(front1.pop(0))
        while n87 and len(pending) >= 4 and (len(pending) > 600 or rng.random() < 0.3):
            chain(4)
            n87 -= 1
        while n84 and pending and (len(pending) > 900 or rng.random() < 0.03):
            chain(1)
            n84 -= 1
    pending.extend(front1)
    while len(pending) >= 4 and n87:
        chain(4)
        n87 -= 1
    while pending:
        chain(1)
    ops.append(69)
    args.append(0)
    return np.array(ops, np.uint64), np.array(args, np.uint64)


def sections(shape=None):
    """[(zxp section, offset, width)] of the fork-9 map"""
    shape = shape or load_shape()
    return [(m["zxp_section"], m["offset"], m["width"]) for m in shape["map"]]
