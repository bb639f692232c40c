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
    challenges 0-3, publics); step42ns draws its columns and constants with
    the reference's locality -- first touches and re-reads at LRU stack
    distances sampled from the "reuse" histogram (tools/bytecode_shape.py),
    so the compiled kernels find as many re-reads in the caches as the
    reference's program would (uniform draws re-read columns ~15x farther
    apart);
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


class _Reuse:
    """Column / constant keys drawn with a program's reuse statistics
    (shape["programs"][name]["reuse"]): a first touch with the reference's
    first-touch fraction, else the key at an LRU stack distance from its
    power-of-two histogram."""

    def __init__(self, stats, rng, new_key, p_first=None):
        self.rng = rng
        self.new_key = new_key  # () -> a key, preferring ones not touched yet
        b = np.array(stats["buckets"], float)
        self.p_first = stats["first"] / (stats["first"] + b.sum()) if p_first is None else p_first
        self.bp = b / b.sum()
        self.stack = []  # most recent last

    def draw(self):
        k = None
        if self.stack and self.rng.random() >= self.p_first:
            b = int(self.rng.choice(len(self.bp), p=self.bp))
            d = 0 if b == 0 else int(self.rng.integers(1 << (b - 1), 1 << b))
            if d < len(self.stack):
                k = self.stack[len(self.stack) - 1 - d]
        if k is None:
            k = self.new_key()
        if k in self.stack:
            self.stack.remove(k)
        self.stack.append(k)
        return k


def generate(name="step42ns", seed=1, shape=None, isa=None, scale=1.0, reserved=None, readable=None):
    """(ops, args) uint64 arrays of a synthetic program shaped like the
    reference's `name` program: step42ns (constraint quotient), step2prev /
    step3prev / step3 (stage-2/3 column programs with shifted stores) or
    step52ns (FRI polynomial); scale < 1 keeps that fraction of every opcode
    count (same mix, same map).  Stage programs inside a proof
    (zkgpu/zkevm_shaped.py): reserved = {section name: columns the program
    must not write}, readable = {section name: the only columns it may read}
    (sections absent from readable: any column); None = no restriction (the
    same program as before for the same seed)."""
    if name == "step42ns":
        return _generate_step42ns(seed, shape, isa, scale)
    if name in ("step2prev", "step3prev", "step3"):
        return _generate_stage(name, seed, shape, isa, scale, reserved, readable)
    if name == "step52ns":
        return _generate_step52ns(seed, shape, isa, scale)
    raise ValueError("unknown program %r" % name)


def _generate_step42ns(seed=1, shape=None, isa=None, scale=1.0):
    """step42ns (the constraint quotient).

    Values form constraint trees: an opcode's temporary operands are taken
    from the not-yet-used values (most recent first), its result joins them;
    the oldest unused values become constraint results once more than
    FRONTIER are waiting, and results are folded into the accumulator by the
    Horner opcodes.  No value is dead, as in the reference."""
    name = "step42ns"
    FRONTIER = 24
    shape = shape or load_shape()
    isa = isa or load_isa()
    table = isa[name]
    rng = np.random.default_rng(seed)
    g = _Gen(name, shape, rng)
    hist = {int(k): max(1, int(round(v * scale))) for k, v in g.sh["opcode_hist"].items()}
    n84, n87 = hist.pop(84, 0), hist.pop(87, 0)
    # columns / constants with the reference's locality (first touches from a
    # shuffled pool per section, then any column of the section's subset)
    pools = {s: list(rng.permutation(g.rcols[s])) for s in g.rsecs}

    def new_col():
        s = g.rsecs[rng.choice(len(g.rsecs), p=g.rprob)]
        c = int(pools[s].pop()) if pools[s] else int(g.rcols[s][rng.integers(len(g.rcols[s]))])
        return (s, c)
    kpool = list(rng.permutation(g.n_const))

    def new_const():
        return int(kpool.pop()) if kpool else int(rng.integers(g.n_const))
    reuse = g.sh.get("reuse")
    # first touches at the rate that reads every column of the reference's
    # distinct sets once over the program's column reads
    n_pool = sum(len(p_) for p_ in pools.values())
    n_reads = scale * sum(g.sh["reads"][s]["accesses"] for s in g.rsecs)
    rcol = _Reuse(reuse, rng, new_col, min(1.0, n_pool / max(n_reads, 1.0))) if reuse else None
    rconst = _Reuse(reuse, rng, new_const) if reuse else None

    def col(dim):
        if rcol is None:
            return g.col(dim)
        s, c = rcol.draw()
        width = g.map[s]["width"]
        return g.map[s]["offset"] + min(c, width - dim), width

    def const():
        return rconst.draw() if rconst else int(rng.integers(g.n_const))
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
        off, w = col(1)
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
                    off, w = col(o[1])
                    put(o[2], off)
                    if k == "P":
                        put(o[3], w)
                    else:
                        put(o[3], g.row_shift)
                        put(o[4], g.dom)
                        put(o[5], w)
                elif k == "K":
                    put(o[2], const())
                elif k == "KS":
                    put(o[2], const())
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


def _find(table, pred):
    """opcodes of `table` whose micro-op list satisfies pred"""
    return [c for c, (_, mops) in sorted(table.items()) if pred(mops)]


def _generate_stage(name, seed=1, shape=None, isa=None, scale=1.0, reserved=None, readable=None):
    """A stage-2/3 column program (step2prev / step3prev / step3,
    zkevm.chelpers.<step>.parser.cpp): the reference's opcode histogram over
    the n-domain sections, every store opcode (86-120) writing a column of
    the program's written set (cm3_n / tmpExp_n, the reference's distinct
    counts), shifted stores (101-119) at the program's row shift.  Hazards are
    those the reference avoids: a written column is never read except the
    cell this row just wrote (store forwarding, same shift), and each written
    column is written at one shift only (no two rows write one cell)."""
    shape = shape or load_shape()
    isa = isa or load_isa()
    table = isa[name]
    rng = np.random.default_rng(seed)
    g = _Gen(name, shape, rng)
    sh = g.sh
    reserved = reserved or {}
    if readable is not None:  # reads only from the readable columns (same subset sizes where they allow)
        for s_ in g.rsecs:
            if s_ in readable:
                ok = np.array(sorted(readable[s_]), np.int64)
                n = min(sh["reads"][s_]["distinct_cols"], ok.size)
                g.rcols[s_] = np.sort(rng.choice(ok, size=n, replace=False)) if n else ok[:0]
    hist = {int(k): max(1, int(round(v * scale))) for k, v in sh["opcode_hist"].items()}
    is_store = lambda c: table[c][1][0][1] is not None and table[c][1][0][1][0] in ("P", "PS")
    stores = {c: n for c, n in hist.items() if is_store(c)}
    body = {c: n for c, n in hist.items() if not is_store(c)}
    # written sets: slots (col, dim) per section, each written at one shift
    wsec = sorted(sh["writes"])
    wprob = np.array([sh["writes"][s_]["accesses"] for s_ in wsec], float)
    wprob /= wprob.sum()
    n3 = sum(n for c, n in stores.items() if table[c][1][0][1][1] == 3)
    n1 = sum(stores.values()) - n3
    slots = {}
    written = {}
    for s_ in wsec:
        width = g.map[s_]["width"]
        res = reserved.get(s_, ())
        want = min(sh["writes"][s_]["distinct_cols"], width - len(res))
        share3 = n3 * 3 / max(1, n1 + 3 * n3)
        k3 = int(want * share3 / 3)
        cols = [c for c in rng.permutation(width) if c not in res] if res else list(rng.permutation(width))
        sl, used = [], set()
        for c in cols:
            if len(sl) >= k3:
                break
            if c + 2 < width and not used & {c, c + 1, c + 2}:
                sl.append([int(c), 3, None])
                used |= {c, c + 1, c + 2}
        for c in cols:
            if len(used) >= want:
                break
            if c not in used:
                sl.append([int(c), 1, None])
                used.add(c)
        slots[s_] = sl
        written[s_] = used
    # reads avoid the written columns
    for s_ in g.rsecs:
        if s_ in written:
            width = g.map[s_]["width"]
            ok = set(range(width)) if readable is None or s_ not in readable else set(readable[s_])
            free = np.array(sorted(ok - written[s_]), np.int64)
            n = min(sh["reads"][s_]["distinct_cols"], free.size)
            g.rcols[s_] = np.sort(rng.choice(free, size=n, replace=False)) if n else free[:0]
    # columns no read may touch (a dim-3 read covers 3 consecutive columns)
    unread = {s_: set(range(g.map[s_]["width"])) - set(readable[s_]) for s_ in (readable or {})}
    cells = []  # written (offset, width, dim, shift) cells, for forwarded reads
    copy1 = _find(table, lambda m: len(m) == 1 and m[0][0] == "copy" and m[0][1][0] == "T1" and m[0][2][0] == "P"
                  and m[0][2][1] == 1)[0]
    mk3 = [c for c in _find(table, lambda m: len(m) == 1 and m[0][1][0] == "T3" and
                            not any(o and o[0] == "T3" for o in m[0][2:]))]
    seq = np.repeat(np.array(list(body), np.int64), list(body.values()))
    st = np.repeat(np.array(list(stores), np.int64), list(stores.values()))
    order = np.concatenate([seq, st])
    rng.shuffle(order)
    # stores after their producers: the first 5 % of the program only computes
    head = max(8, len(order) // 20)
    order = list(order)
    first = [c for c in order[:head] if not is_store(c)] + [c for c in order[:head] if is_store(c)]
    order = first + order[head:]
    ops, args = [], []
    n1s, n3s = g.n1, g.n3
    w1, w3 = [], []  # temp slots written so far
    front1 = []
    free1 = list(range(n1s))

    def read_col(s_, dim):
        """a column (dim 1) or 3 consecutive columns (dim 3) none of which the
        program writes, from section s_ (another section if s_ has none)"""
        for s2 in [s_] + [x for x in g.rsecs if x != s_]:
            cols = g.rcols[s2]
            if not len(cols):
                continue
            width = g.map[s2]["width"]
            bad = written.get(s2, set()) | unread.get(s2, set())
            for _ in range(64):
                c = int(cols[rng.integers(len(cols))])
                c = min(c, width - dim)
                if not bad & set(range(c, c + dim)):
                    return g.map[s2]["offset"] + c, width
        raise AssertionError("no readable columns")

    def emit(code, pick_dst3=None):
        nargs, mops = table[int(code)]
        a = [0] * nargs
        filled = [False] * nargs

        def put(f, v):
            if f >= 0 and not filled[f]:
                a[f] = int(v)
                filled[f] = True

        for (op, d, x, y) in mops:
            for o in (x, y):
                if o is None:
                    continue
                k = o[0]
                if k == "T1" and not filled[o[2]]:
                    if front1 and rng.random() < 0.85:
                        put(o[2], front1.pop(len(front1) - 1 - min(int(rng.exponential(2)), len(front1) - 1)))
                    else:
                        put(o[2], w1[len(w1) - 1 - min(int(rng.exponential(8)), len(w1) - 1)])
                elif k == "T3" and not filled[o[2]]:
                    put(o[2], w3[int(rng.integers(len(w3)))])
                elif k in ("P", "PS"):
                    s_ = g.rsecs[rng.choice(len(g.rsecs), p=g.rprob)]
                    fw = [cl for cl in cells if cl[2] == o[1] and (cl[3] != 0) == (k == "PS")]
                    fw_s = [cl for cl in fw if cl[4] == s_]
                    if fw and (rng.random() < 0.05 or (len(g.rcols[s_]) == 0 and fw_s)):
                        # a cell this row wrote (the same shift): forwarded
                        cl = (fw_s or fw)[int(rng.integers(len(fw_s or fw)))]
                        off, w = cl[0], cl[1]
                    else:
                        off, w = read_col(s_, o[1])
                    put(o[2], off)
                    if k == "P":
                        put(o[3], w)
                    else:
                        put(o[3], g.row_shift)
                        put(o[4], g.dom)
                        put(o[5], w)
                elif k in ("K", "KS"):
                    put(o[2], rng.integers(g.n_const))
                    if k == "KS":
                        put(o[3], g.row_shift)
                        put(o[4], g.dom)
                elif k == "L":
                    put(o[2], int(rng.integers(0, P, dtype=np.uint64)) if rng.random() < 0.3
                        else int(rng.integers(0, 64)))
                elif k == "C":
                    put(o[2], g.chal[rng.integers(len(g.chal))])
                elif k == "U":
                    put(o[2], 0)
            kd = d[0]
            if kd == "T1" and not filled[d[2]]:
                s_ = free1.pop(0) if free1 else w1[int(rng.integers(len(w1)))]
                put(d[2], s_)
                if s_ not in w1:
                    w1.append(s_)
                front1.append(s_)
                del front1[:-24]
            elif kd == "T3" and not filled[d[2]]:
                s_ = pick_dst3 if pick_dst3 is not None else int(rng.integers(n3s))
                put(d[2], s_)
                if s_ not in w3:
                    w3.append(s_)
            elif kd in ("P", "PS") and not filled[d[2]]:
                shift = 0 if kd == "P" else g.row_shift
                for _ in range(1000):
                    s_ = wsec[rng.choice(len(wsec), p=wprob)]
                    cand = [x for x in slots[s_] if x[1] == d[1] and x[2] in (None, shift)]
                    if cand:
                        break
                x = cand[int(rng.integers(len(cand)))]
                x[2] = shift
                width = g.map[s_]["width"]
                off = g.map[s_]["offset"] + x[0]
                put(d[2], off)
                if kd == "P":
                    put(d[3], width)
                else:
                    put(d[3], g.row_shift)
                    put(d[4], g.dom)
                    put(d[5], width)
                cells.append((off, width, d[1], shift, s_))
        assert all(filled), (code, mops, filled)
        ops.append(int(code))
        args.extend(a)

    for _ in range(4):  # values first: every temporary an op reads is written earlier in the row
        emit(copy1)
    for j in range(n3s):
        emit(mk3[int(rng.integers(len(mk3)))], pick_dst3=j)
    for code in order:
        emit(code)
    return np.array(ops, np.uint64), np.array(args, np.uint64)


def _generate_step52ns(seed=1, shape=None, isa=None, scale=1.0):
    """The FRI polynomial (step52ns, zkevm.chelpers.step52ns.parser.cpp):
    a Horner chain with v1 over every committed column (opcodes 0 / 16 / 17),
    saved (3); Horner chains with v2 over (pol - eval) for the evaluations
    (21 / 18 / 19 / 20) times xDivXSubXi (5), then the primed group times
    xDivXSubWXi (6), summed (8), stored to f_2ns (15).  Counts follow the
    reference's histogram; columns from the fork-9 2ns sections, each once
    per chain, eval indices distinct."""
    shape = shape or load_shape()
    isa = isa or load_isa()
    table = isa["step52ns"]
    rng = np.random.default_rng(seed)
    g = _Gen("step52ns", shape, rng)
    h = {int(k): v for k, v in g.sh["opcode_hist"].items()}
    sc = lambda c: max(1, int(round(h.get(c, 1) * scale)))
    ops, args = [], []

    def emit(code, *a):
        assert len(a) == table[code][0], (code, a)
        ops.append(code)
        args.extend(int(x) for x in a)

    # committed columns, each once: dim-1 (16) and dim-3 (17) terms
    cols1, cols3 = [], []
    for s_ in g.rsecs:
        m = g.map[s_]
        w = m["width"]
        cs = list(rng.permutation(w))
        k3 = min(sc(17) * w // max(1, sum(g.map[x]["width"] for x in g.rsecs)), w // 3)
        used = set()
        for c in cs:
            if len([x for x in cols3 if x[2] == s_]) >= k3:
                break
            if c + 2 < w and not used & {c, c + 1, c + 2}:
                cols3.append((m["offset"] + int(c), w, s_))
                used |= {c, c + 1, c + 2}
        cols1 += [(m["offset"] + int(c), w, s_) for c in cs if c not in used]
    rng.shuffle(cols1)
    rng.shuffle(cols3)
    cols1 = cols1[:sc(16) + 1]
    cols3 = cols3[:sc(17)]
    emit(0, cols1[0][0], cols1[0][1])  # A0 = P * v1
    terms = [(16, c) for c in cols1[1:]] + [(17, c) for c in cols3]
    rng.shuffle(terms)
    for code, c in terms:
        emit(code, c[0], c[1])  # A0 = A0 * v1 + P
    emit(3)  # A1 = A0 * v1
    n_ev = min(int(g.sh["n_evals_used"] or 1972), 1 + int(round(1972 * scale)))
    evs = list(rng.permutation(max(n_ev, 4)))
    groups = [(5, evs[:len(evs) * 2 // 3]), (6, evs[len(evs) * 2 // 3:])]  # unprimed x xdiv, primed x xdivw
    for gi, (xop, ev) in enumerate(groups):
        if gi:
            emit(3)  # A1 = A0 * v1 (the running sum, saved)
        c = cols1[int(rng.integers(len(cols1)))]
        emit(21, c[0], c[1], ev[0])  # A0 = P - E
        for e in ev[1:]:
            r = rng.random()
            if r < 0.71:
                c = cols1[int(rng.integers(len(cols1)))]
                emit(18, c[0], c[1], e)  # A0 = A0 * v2 + (P - E)
            elif r < 0.88:
                emit(19, int(rng.integers(g.n_const)), e)  # A0 = A0 * v2 + (K - E)
            else:
                c = cols3[int(rng.integers(len(cols3)))] if cols3 else cols1[0]
                emit(20, c[0], c[1], e)  # A0 = A0 * v2 + (P3 - E)
        emit(xop)  # A0 *= xDivXSubXi / xDivXSubWXi
        emit(8)  # A0 = A1 + A0
    emit(15)  # f_2ns = A0
    return np.array(ops, np.uint64), np.array(args, np.uint64)


def sections(shape=None):
    """[(zxp section, offset, width)] of the fork-9 map"""
    shape = shape or load_shape()
    return [(m["zxp_section"], m["offset"], m["width"]) for m in shape["map"]]
