#!/usr/bin/env python3
"""Column-affinity partition of the quotient program, simulated before
building it (VERDICT r5 "next" 4: "simulate a column-affinity partition of the
program into segments -- minimise the distinct columns per segment plus the
carries -- with the Belady tool").  Build container, no GPU.

Input: step42ns compiled by the product's host compiler (zkgpu_zxp_compile,
as the bench's quotient runs it): the step42ns-shaped synthetic program
(zkgpu/synthetic_bytecode.py, seed 1) and, when /root/reference is present,
the reference's own fork-9 step42ns bytecode (read at run time, nothing of it
stored; tools/parser_isa.py).  Per row, the kernel's column reads in program
order (a COL3 operand is three column reads, a DOT term one); temporaries are
SSA values, so the instruction list is a DAG and any topological order of it
computes the same row.

Partitions compared (each into S segments of equal VALU estimate,
zxp_segment.cpp zxp_instr_cost):
  contiguous  -- the product's cut (zxp_segment: consecutive instructions,
                 cut where the fewest words are live);
  affinity    -- list scheduling that grows one segment at a time, always
                 taking the ready instruction (all operands defined) that
                 adds the fewest new columns to the segment's column set
                 (ties: program order) -- the greedy minimiser of distinct
                 columns per segment; values read by a later segment are
                 carried through scratch columns (one store + reads);
  affinity+lru -- the same, the tie broken toward the columns read most
                 recently.
For each: distinct columns per segment (summed), carried words, and the HBM
column reads per row the kernel would make with a Belady LDS cache of k
slots per lane per segment (lds_column_cache's rule: evict the value read
furthest in the future, bypass when the new one is read later still;
k = 12 is today's kernel, 32 / 48 what 2 waves per SIMD could hold),
carried values' reads included.  The quotient's target (<= 4.5x
the algorithmic bytes) is ~6,600 such reads per row on the shaped program.

Usage: tools/s42_partition_sim.py [--segments S] [--real] [out.json]
"""
import json
import os
import sys
from heapq import heappop, heappush

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd"), os.path.join(ROOT, "tools")]

TMP1, TMP3, COL, COL3 = 0, 1, 2, 3
DOT1, DOT3, COPY, MUL = 4, 5, 3, 2
SCRATCH = 1 << 20
INF = 1 << 62


def compiled(kind):
    import zkgpu
    from real_programs_compile import consts, program
    prog, _ = program(kind, "step42ns")
    return zkgpu.zxp_compile(prog, *consts())


def dim(o):
    return 3 if o[0] in (TMP3, COL3) or (o[0] == 12 and o[2] == 3) or o[0] in (5, 8, 9, 10) else 1


def analyse(cp):
    """per instruction: column keys read (in order), temps read, temp defined, cost"""
    ins, opn, term = cp["instr"], cp["opnd"], cp["term"]
    reads, tdeps, cost = [], [], []
    for k in range(ins.shape[0]):
        op, dst, a, b = (int(v) for v in ins[k])
        cols, deps = [], []

        def use(o, comp=None):
            kind, x, y, z = (int(v) for v in opn[o])
            if kind == COL:
                cols.append((x, y, z))
            elif kind == COL3:
                for j in ((comp,) if comp is not None else range(3)):
                    cols.append((x, y + j, z))
            elif kind in (TMP1, TMP3):
                deps.append(o)

        if op in (DOT1, DOT3):
            n = 0
            for t in range(a, a + b):
                s = int(term["src"][t])
                if s != 0xFFFFFFFF:
                    use(s, int(term["comp"][t]) if int(opn[s][0]) == COL3 else None)
                    n += 1
            c = 30 + 20 * n if op == DOT3 else 10 + 7 * n
        else:
            use(a)
            if op != COPY:
                use(b)
            da, db = dim(opn[a]), dim(opn[b])
            c = 1 if op == COPY else ((160 if da == 3 and db == 3 else 66 if 3 in (da, db) else 22) if op == MUL
                                      else 7 * max(da, db))
        reads.append(cols)
        tdeps.append(deps)
        cost.append(c)
    defs = [int(ins[k][1]) if int(opn[int(ins[k][1])][0]) in (TMP1, TMP3) else -1 for k in range(ins.shape[0])]
    return reads, tdeps, defs, cost


def belady(stream, slots):
    """misses of a Belady cache of `slots` values over one segment's reads"""
    nx = [INF] * len(stream)
    last = {}
    for r in range(len(stream) - 1, -1, -1):
        nx[r] = last.get(stream[r], INF)
        last[stream[r]] = r
    cache = {}  # key -> next use
    heap = []  # (-next use, key) lazy
    miss = 0
    for r, key in enumerate(stream):
        if key in cache:
            cache[key] = nx[r]
            if nx[r] == INF:
                del cache[key]
            else:
                heappush(heap, (-nx[r], key))
            continue
        miss += 1
        if nx[r] == INF:
            continue
        if len(cache) >= slots:
            while True:  # furthest next use (skip stale heap entries)
                nu, kk = heap[0]
                if kk in cache and cache[kk] == -nu:
                    break
                heappop(heap)
            if -heap[0][0] <= nx[r]:
                continue  # bypass
            _, kk = heappop(heap)
            del cache[kk]
        cache[key] = nx[r]
        heappush(heap, (-nx[r], key))
    return miss


def evaluate(order_segs, reads, tdeps, defs, slots_list):
    """order_segs: list of instruction lists (each a valid order).  Carried
    temps: defined in one segment, read in a later one (a store, then a
    scratch column read per reading segment's first-use, cached like columns)."""
    seg_of = {}
    for s, seg in enumerate(order_segs):
        for k in seg:
            seg_of[k] = s
    def_seg = {}
    for k, d in enumerate(defs):
        if d >= 0:
            def_seg[d] = seg_of[k]
    carried = set()
    streams = []
    distinct = 0
    for s, seg in enumerate(order_segs):
        st = []
        for k in seg:
            st.extend(reads[k])
            for d in tdeps[k]:
                if def_seg[d] < s:
                    st.append((SCRATCH, d, 0))
                    carried.add(d)
        streams.append(st)
        distinct += len(set(st))
    out = {"segments": len(order_segs), "distinct_cols_per_segment_sum": distinct,
           "carried_values": len(carried), "reads_per_row": sum(len(x) for x in streams)}
    for sl in slots_list:
        out["hbm_reads_%d_slots" % sl] = sum(belady(st, sl) for st in streams)
    out["stores_per_row_carries"] = len(carried)
    return out


def contiguous(n, cost, nseg):
    tot = sum(cost)
    segs, cur, acc, q = [], [], 0, 1
    for k in range(n):
        cur.append(k)
        acc += cost[k]
        if q < nseg and acc >= tot * q / nseg:
            segs.append(cur)
            cur, q = [], q + 1
    segs.append(cur)
    return [s for s in segs if s]


def affinity(reads, tdeps, defs, cost, nseg, recency=False):
    n = len(reads)
    def_of = {d: k for k, d in enumerate(defs) if d >= 0}
    preds = [set(def_of[d] for d in tdeps[k]) for k in range(n)]
    succ = [[] for _ in range(n)]
    for k in range(n):
        for p in preds[k]:
            succ[p].append(k)
    indeg = [len(p) for p in preds]
    ready = set(k for k in range(n) if indeg[k] == 0)
    tot = sum(cost)
    segs, q = [], 1
    done = 0
    cur, cols, acc, lastuse, clock = [], set(), 0, {}, 0
    while ready:
        best, bk = None, None
        for k in ready:
            new = sum(1 for c in set(reads[k]) if c not in cols)
            rec = -max((lastuse.get(c, -1) for c in reads[k]), default=-1) if recency else 0
            key = (new, rec, k)
            if bk is None or key < bk:
                bk, best = key, k
        ready.discard(best)
        cur.append(best)
        for c in reads[best]:
            cols.add(c)
            lastuse[c] = clock
        clock += 1
        acc += cost[best]
        done += 1
        for s2 in succ[best]:
            indeg[s2] -= 1
            if indeg[s2] == 0:
                ready.add(s2)
        if q < nseg and acc >= tot * q / nseg:
            segs.append(sorted(cur))
            cur, cols, q = [], set(), q + 1
    if cur:
        segs.append(sorted(cur))
    assert done == n, "dependency cycle"
    return segs


def refine(segs, reads, tdeps, defs, cost, opn, passes=6, slack=0.15):
    """local search from a partition: move single instructions to the
    neighbouring segment while dependencies allow it, the segment stays within
    (1 + slack) of the mean VALU estimate, and distinct columns per segment
    plus carried words (a store and a read per later reading segment) fall"""
    from collections import Counter, defaultdict
    n = len(reads)
    S = len(segs)
    seg = [0] * n
    for s, g in enumerate(segs):
        for k in g:
            seg[k] = s
    def_of = {d: k for k, d in enumerate(defs) if d >= 0}
    preds = [set(def_of[d] for d in tdeps[k]) for k in range(n)]
    succ = [[] for _ in range(n)]
    for k in range(n):
        for p_ in preds[k]:
            succ[p_].append(k)
    readers = defaultdict(list)  # value -> reading instructions
    for k in range(n):
        for d in set(tdeps[k]):
            readers[d].append(k)
    wdim = {d: dim(opn[d]) for d in readers}
    colcnt = [Counter() for _ in range(S)]
    for k in range(n):
        for c in set(reads[k]):
            colcnt[seg[k]][c] += 1
    load = [0] * S
    for k in range(n):
        load[seg[k]] += cost[k]
    cap = (1 + slack) * sum(cost) / S

    def carry(d):
        sd = seg[def_of[d]]
        later = set(seg[r] for r in readers[d] if seg[r] > sd)
        return (1 + len(later)) * wdim[d] if later else 0

    moved = 0
    for _ in range(passes):
        changed = 0
        for k in range(n):
            s = seg[k]
            for t in (s - 1, s + 1):
                if t < 0 or t >= S or load[t] + cost[k] > cap:
                    continue
                if t < s and any(seg[p_] > t for p_ in preds[k]):
                    continue
                if t > s and any(seg[q] < t for q in succ[k]):
                    continue
                cols = set(reads[k])
                dcol = sum((colcnt[t][c] == 0) - (colcnt[s][c] == 1) for c in cols)
                vals = set(tdeps[k]) | ({defs[k]} if defs[k] in readers else set())
                before = sum(carry(d) for d in vals)
                seg[k] = t
                after = sum(carry(d) for d in vals)
                gain = dcol + after - before
                if gain < 0:
                    for c in cols:
                        colcnt[s][c] -= 1
                        if colcnt[s][c] == 0:
                            del colcnt[s][c]
                        colcnt[t][c] += 1
                    load[s] -= cost[k]
                    load[t] += cost[k]
                    changed += 1
                    break
                seg[k] = s
        moved += changed
        if not changed:
            break
    out = [[] for _ in range(S)]
    for k in range(n):
        out[seg[k]].append(k)
    return [g for g in out if g], moved


def main():
    nseg = int(sys.argv[sys.argv.index("--segments") + 1]) if "--segments" in sys.argv else 0
    kinds = ["synthetic"] + (["real"] if "--real" in sys.argv and os.path.isdir("/root/reference") else [])
    outp = [a for a in sys.argv[1:] if a.endswith(".json")]
    slots = (12, 16, 32, 48)
    doc = {"what": __doc__.split("\n\n")[0].strip(), "generated_by": "tools/s42_partition_sim.py", "programs": {}}
    for kind in kinds:
        cp = compiled(kind)
        reads, tdeps, defs, cost = analyse(cp)
        n = len(reads)
        S = nseg or max(1, (sum(cost) + 25000) // 50000)  # zxp_jit.hip segments_for
        distinct = len(set(c for r in reads for c in r))
        res = {"instructions": n, "segments": S, "distinct_cols_program": distinct,
               "col_reads_per_row": sum(len(r) for r in reads)}
        print(kind, res, flush=True)
        for name, segs in (("one_segment", [list(range(n))]),
                           ("contiguous", contiguous(n, cost, S)),
                           ("affinity", affinity(reads, tdeps, defs, cost, S)),
                           ("affinity_lru", affinity(reads, tdeps, defs, cost, S, recency=True))):
            res[name] = evaluate(segs, reads, tdeps, defs, slots)
            print(" ", name, res[name], flush=True)
        for slack in (0.15, 0.5):
            segs, moved = refine(contiguous(n, cost, S), reads, tdeps, defs, cost, cp["opnd"], slack=slack)
            name = "contiguous_refined_slack%g" % slack
            res[name] = evaluate(segs, reads, tdeps, defs, slots)
            res[name]["moves"] = moved
            print(" ", name, res[name], flush=True)
        doc["programs"][kind] = res
    if outp:
        with open(outp[0], "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
