#!/usr/bin/env python3
"""Summary statistics of the reference's zkEVM Steps bytecode (the shape, not
the program): per program the op / arg counts, temporaries, opcode histogram,
the columns it reads and writes per section of the fork-9 memory map (SURVEY.md
Appendix B), row shifts, and the challenge / public / eval indices it uses.

The bytecode itself (op*/args* in zkevm.chelpers.<step>.parser.hpp) is read
from /root/reference and never stored; the statistics go to
tests/golden/zkevm_bytecode_shape.json, from which
zkgpu/synthetic_bytecode.py builds programs of the same shape for the GPU
tests and the step42ns bench (the GPU box has no reference tree).

The column reads' locality is kept as a statistic too ("reuse"): in
program order, every read of a column (memory-map section or constant) is
either a first touch or a re-read at some LRU stack distance (the number of
distinct columns read since this one was last read).  The histogram of those
distances, in power-of-two buckets, lets the generator reproduce how closely
the reference's programs cluster their re-reads -- which decides how many of
the compiled kernels' column loads hit the L2.

Usage: tools/bytecode_shape.py [out.json]
"""
import collections
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import parser_isa  # noqa: E402

# ZXP section, mapOffsets, mapSectionsN
MAP = [("cm1_n", 0, 0, 751), ("cm2_n", 1, 6299844608, 168), ("cm3_n", 2, 7709130752, 408),
       ("tmpExp_n", 3, 11182014464, 389), ("cm1_2ns", 5, 14445182976, 751), ("cm2_2ns", 6, 27044872192, 168),
       ("cm3_2ns", 7, 29863444480, 408), ("cm4_2ns", 8, 36708548608, 6)]


def section_of(off, stride):
    for name, sec, base, w in MAP:
        if w == stride and base <= off < base + w:
            return name, off - base
    raise ValueError((off, stride))


class Lru:
    """LRU stack of keys: access(k) -> stack distance (None on first touch)"""

    def __init__(self):
        self.stack = []  # most recent last

    def access(self, k):
        try:
            i = self.stack.index(k)
        except ValueError:
            self.stack.append(k)
            return None
        d = len(self.stack) - 1 - i
        self.stack.pop(i)
        self.stack.append(k)
        return d


def reuse_hist(dists, first):
    """{"first": first touches, "buckets": counts of d in [0], [1], [2, 3], [4, 7], ...}"""
    b = [0] * 16
    for d in dists:
        b[min(15, d.bit_length())] += 1
    while b and b[-1] == 0:
        b.pop()
    return {"first": first, "buckets": b}


def shape(name, isa):
    ops, args = parser_isa.load_bytecode(name)
    table = isa[name]
    sizes = parser_isa.header_sizes()[name]
    hist = collections.Counter(int(o) for o in ops)
    reads = collections.defaultdict(collections.Counter)
    writes = collections.defaultdict(collections.Counter)
    shifts, moduli = collections.Counter(), collections.Counter()
    chal, pub, ev, kcols = collections.Counter(), set(), set(), set()
    lru, dists, first = Lru(), [], 0

    def touch(key):
        nonlocal first
        d = lru.access(key)
        if d is None:
            first += 1
        else:
            dists.append(d)
    ia = 0
    for o in ops:
        e = table[int(o)]
        for (op, d, a, b) in e["ops"]:
            for role, x in (("w", d), ("r", a), ("r", b)):
                if not x:
                    continue
                k = x[0]
                if k in ("P", "PS"):
                    off, stride = int(args[ia + x[2]]), int(args[ia + x[-1]])
                    sec, col = section_of(off, stride)
                    for c in range(x[1]):
                        (writes if role == "w" else reads)[sec][col + c] += 1
                    if role == "r":
                        touch((sec, col))
                    if k == "PS":
                        shifts[int(args[ia + x[3]])] += 1
                        moduli[int(args[ia + x[4]])] += 1
                elif k in ("K", "KS"):
                    kcols.add(int(args[ia + x[1]]))
                    touch(("const", int(args[ia + x[1]])))
                    if k == "KS":
                        shifts[int(args[ia + x[2]])] += 1
                        moduli[int(args[ia + x[3]])] += 1
                elif k == "C":
                    chal[int(args[ia + x[1]])] += 1
                elif k == "U":
                    pub.add(int(args[ia + x[1]]))
                elif k == "E":
                    ev.add(int(args[ia + x[1]]))
        ia += e["nargs"]
    assert ia == len(args)
    return {
        "n_ops": int(len(ops)), "n_args": int(len(args)),
        "ntemp1": sizes.get("NTEMP1", 0), "ntemp3": sizes.get("NTEMP3", 0),
        "opcode_hist": {str(k): v for k, v in sorted(hist.items())},
        "reads": {s: {"distinct_cols": len(c), "accesses": sum(c.values())} for s, c in sorted(reads.items())},
        "writes": {s: {"distinct_cols": len(c), "accesses": sum(c.values())} for s, c in sorted(writes.items())},
        "row_shifts": {str(k): v for k, v in sorted(shifts.items())},
        "moduli": {str(k): v for k, v in sorted(moduli.items())},
        "challenges": {str(k): v for k, v in sorted(chal.items())},
        "max_public": max(pub) if pub else None, "n_evals_used": len(ev), "max_eval": max(ev) if ev else None,
        "const_cols": len(kcols),
        "reuse": reuse_hist(dists, first),
    }


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(HERE), "tests", "golden",
                                                              "zkevm_bytecode_shape.json")
    isa = parser_isa.extract()
    doc = {"_doc": "statistics of the fork-9 zkEVM Steps bytecode (tools/bytecode_shape.py over "
                   "src/starkpil/zkevm/chelpers/zkevm.chelpers.<step>.parser.hpp); no program content",
           "map": [{"section": n, "zxp_section": s, "offset": o, "width": w} for n, s, o, w in MAP],
           "n_const": 234, "n_bits": 23, "n_bits_ext": 24,
           "programs": {name: shape(name, isa) for name in parser_isa.PARSERS}}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for name, s in doc["programs"].items():
        print(name, s["n_ops"], s["n_args"], s["reads"], s["writes"], s["row_shifts"], s["challenges"])


if __name__ == "__main__":
    main()
