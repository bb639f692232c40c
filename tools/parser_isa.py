#!/usr/bin/env python3
"""Extract the instruction set of the reference's Steps bytecode interpreters.

The zkEVM constraint/expression code is bytecode (`op*[]` opcodes, `args*[]`
operands, `src/starkpil/zkevm/chelpers/zkevm.chelpers.<step>.parser.hpp`)
evaluated by an AVX2 interpreter: one `case` per opcode in
`ZkevmSteps::<step>_parser_first_avx` (`…<step>.parser.cpp`, e.g.
step42ns.parser.cpp:24-784, step52ns.parser.cpp:9-226).  This tool reads those
`case` tables AS TEXT and restates each opcode as a list of micro-operations

    (op, dst, a, b)       op in add / sub / mul / copy / qout

over operands

    ("T1", k)               tmp1[args[k]]            base temporary
    ("T3", k)               tmp3[args[k]]            F_p^3 temporary
    ("P", d, o, s)          pols[args[o] + i*args[s]]              (d = 1 or 3 columns)
    ("PS", d, o, h, m, s)   pols[args[o] + ((i+args[h]) % args[m])*args[s]]
    ("K", k)                constPols(args[k], i)
    ("KS", k, h, m)         constPols(args[k], (i+args[h]) % args[m])
    ("KL", c)               constPols(c, i), c a literal column (step52ns)
    ("L", k)                Goldilocks literal args[k]
    ("C", k) / ("CL", c)    challenges[args[k]] / challenges[c]
    ("U", k)                publicInputs[args[k]]
    ("E", k) / ("EL", e)    evals[args[k]] / evals[e]                (step52ns)
    ("X",) ("ZI",) ("XDIV",) ("XDIVW",) ("Q",) ("F",)
    ("A", n)                step52ns F_p^3 accumulator tmp<n> (zero at row start for n = 2)

with k the argument index relative to the opcode's first argument.  The
micro-operation semantics are the Goldilocks / Goldilocks3 functions named in
the case body: dst = a (op) b, result dimension max(dim a, dim b), F_p^3
products in F_p[x]/(x^3 - x - 1); `qout` is q_2ns[i] = zhInv(i) * a.

The output is the ISA table the product converter (zkevm-prover_amd/csrc/
parser_convert.cpp, via the generated csrc/parser_isa.inc) and the CPU oracle
(oracle/parser.c) follow; tests/test_parser_isa.py re-extracts it from
/root/reference and requires it to equal the committed table.  The
bytecode arrays themselves are never copied into the repository.

Usage: tools/parser_isa.py [--reference DIR] [--emit-inc PATH] [--json PATH]
"""
import argparse
import json
import os
import re
import sys

REF = "/root/reference/src/starkpil/zkevm/chelpers"
PARSERS = ["step2prev", "step3prev", "step3", "step42ns", "step52ns"]


def split_args(s):
    out, depth, cur = [], 0, ""
    for c in s:
        if c in "([":
            depth += 1
        elif c in ")]":
            depth -= 1
        if c == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += c
    if cur.strip():
        out.append(cur.strip())
    return out


def function_body(text, name):
    m = re.search(r"void ZkevmSteps::%s\(StepsParams &params, uint64_t nrows, uint64_t nrowsBatch\)\s*\{" % name,
                  text)
    if not m:
        raise KeyError(name)
    depth, j = 1, m.end()
    while depth:
        c = text[j]
        depth += (c == "{") - (c == "}")
        j += 1
    return text[m.end():j - 1]


def cases(body):
    """{opcode: case body text} of the dispatch switch (comments stripped)."""
    body = re.sub(r"//[^\n]*", "", body)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    parts = re.split(r"\bcase (\d+):", body)
    out = {}
    for k in range(1, len(parts), 2):
        txt = parts[k + 1]
        # the case ends at its `break;` (fused opcodes have several i_args += in between)
        end = txt.find("break;")
        out[int(parts[k])] = txt[:end] if end >= 0 else txt
    return out


A = r"args\w*\[i_args(?: \+ (\d+))?\]"


def aidx(s, base):
    m = re.fullmatch(r"\(?" + A + r"\)?", s.strip())
    if not m:
        raise ValueError("not an argument reference: %r" % s)
    return base + int(m.group(1) or 0)


def parse_offsets(expr, base):
    """offsetsN[j] = ... -> operand template (without dim)"""
    e = expr.strip()
    m = re.fullmatch(A + r" \+ \(\(\(i \+ j\) \+ " + A + r"\) % " + A + r"\) \* " + A, e)
    if m:
        g = [base + int(x or 0) for x in m.groups()]
        return ("PS", g[0], g[1], g[2], g[3])
    m = re.fullmatch(A + r" \+ \(\(\(i \+ j\) \+ " + A + r"\) % " + A + r"\) \* numpols", e)
    if m:
        g = [base + int(x or 0) for x in m.groups()]
        return ("KS", g[0], g[1], g[2])
    m = re.fullmatch(A + r" \+ \(i \+ j\) \* " + A, e)
    if m:
        g = [base + int(x or 0) for x in m.groups()]
        return ("P", g[0], g[1])
    m = re.fullmatch(A + r" \+ \(i \+ j\) \* numpols", e)
    if m:
        return ("K", base + int(m.group(1) or 0))
    if re.fullmatch(r"FIELD_EXTENSION \* \(j \+ AVX_SIZE_ \* " + A + r"\)", e):
        return ("IGNORE",)
    raise ValueError("offsets expression: %r" % e)


def dims_of(fn):
    """operand dimensions (a, b) from the Goldilocks3 function name: add13c -> (1, 3)"""
    m = re.fullmatch(r"(add|sub|mul|mult|copy)(\d?c?)(\d?c?)", fn)
    if not m:
        raise ValueError(fn)
    da = int(m.group(2)[0]) if m.group(2) else 3
    db = int(m.group(3)[0]) if m.group(3) else 3
    return m.group(1), da, db


def classify(arg, base, pending_placeholder):
    """one call argument -> operand tuple, None (stride / skipped) or placeholder marker"""
    s = arg.strip()
    s = re.sub(r"^\(Goldilocks3?::Element\s*&\)\s*\*?", "", s).strip()
    if re.fullmatch(r"tmp1\[\(?" + A + r"\)?\]", s):
        return ("T1", aidx(s[5:-1], base))
    if re.fullmatch(r"tmp3\[\(?" + A + r"\)?\]", s):
        return ("T3", aidx(s[5:-1], base))
    m = re.fullmatch(r"&params\.pols\[" + A + r" \+ i \* " + A + r"\]", s)
    if m:
        return ("P", base + int(m.group(1) or 0), base + int(m.group(2) or 0))
    if s == "&params.pols[0]":
        return ("PH_P",)
    m = re.fullmatch(r"&params\.pConstPols(?:2ns)?->getElement\(" + A + r", i\)", s)
    if m:
        return ("K", base + int(m.group(1) or 0))
    if re.fullmatch(r"&params\.pConstPols(?:2ns)?->getElement\(0, 0\)", s):
        return ("PH_K",)
    m = re.fullmatch(r"&params\.pConstPols2ns->getElement\((\d+), i\)", s)
    if m:
        return ("KL", int(m.group(1)))
    m = re.fullmatch(r"Goldilocks::fromU64\(" + A + r"\)", s)
    if m:
        return ("L", base + int(m.group(1) or 0))
    m = re.fullmatch(r"params\.challenges\[" + A + r"\]", s)
    if m:
        return ("C", base + int(m.group(1) or 0))
    m = re.fullmatch(r"params\.challenges\[(\d+)\]", s)
    if m:
        return ("CL", int(m.group(1)))
    m = re.fullmatch(r"params\.publicInputs\[" + A + r"\]", s)
    if m:
        return ("U", base + int(m.group(1) or 0))
    if re.fullmatch(r"params\.x_(n|2ns)\[i\]", s):
        return ("X",)
    m = re.fullmatch(r"offsets(\d)", s)
    if m:
        return ("OFF", int(m.group(1)))
    # stride arguments carry no math
    if re.fullmatch(r"\(?" + A + r"\)?", s) or s in ("numpols", "FIELD_EXTENSION") or \
            re.fullmatch(r"params\.x_(n|2ns)\.offset\(\)", s) or s == "params.pConstPols2ns->numPols()":
        return None
    # step52ns
    m = re.fullmatch(r"&evals_\[" + A + r" \* 3\]", s)
    if m:
        return ("E", base + int(m.group(1) or 0))
    if s == "evals_":
        return ("EL", 0)
    if s == "params.xDivXSubXi[i]":
        return ("XDIV",)
    if s == "params.xDivXSubWXi[i]":
        return ("XDIVW",)
    if s == "&(params.f_2ns[i * 3])":
        return ("F",)
    m = re.fullmatch(r"tmp(\d)_(\d)", s)
    if m:
        return ("ACC", int(m.group(1)), int(m.group(2)))
    m = re.fullmatch(r"chall(\d)(o?)(\d)_", s)
    if m:
        return ("CHP", int(m.group(1)), m.group(2), int(m.group(3)))
    raise ValueError("unsupported argument %r" % s)


def statement_ops(stmt, base, offsets):
    """a call statement -> list of micro-operations"""
    m = re.fullmatch(r"(Goldilocks3?)::(\w+?)(?:_avx)?\((.*)\)", stmt, re.S)
    if not m:
        raise ValueError("statement %r" % stmt[:160])
    cls, fn, argtxt = m.group(1), m.group(2), m.group(3)
    ops = []
    raw = [classify(a, base, None) for a in split_args(argtxt)]
    raw = [r for r in raw if r is not None]
    # group step52ns accumulator / challenge triples
    grouped = []
    k = 0
    while k < len(raw):
        r = raw[k]
        if r[0] == "ACC":
            assert r[2] == 0 and raw[k + 1] == ("ACC", r[1], 1) and raw[k + 2] == ("ACC", r[1], 2), raw
            grouped.append(("A", r[1]))
            k += 3
        elif r[0] == "CHP":
            # chall<c>0_ chall<c>1_ chall<c>2_ chall<c>o0_ ... = challenges[c] (+ its Karatsuba sums)
            c = r[1]
            assert all(x[0] == "CHP" and x[1] == c for x in raw[k:k + 6]), raw
            grouped.append(("CL", c))
            k += 6
        else:
            grouped.append(r)
            k += 1
    # bind &pols[0] / getElement(0,0) placeholders to the offsets arrays, in order
    ph = [i for i, r in enumerate(grouped) if r[0] in ("PH_P", "PH_K")]
    offs = [r for r in grouped if r[0] == "OFF"]
    if len(ph) != len(offs):
        raise ValueError("placeholders %s vs offsets %s in %r" % (ph, offs, stmt[:120]))
    for i, o in zip(ph, offs):
        t = offsets[o[1]]
        if grouped[i][0] == "PH_K":
            if t[0] not in ("KS", "K"):
                raise ValueError("const placeholder bound to %s" % (t,))
        elif t[0] not in ("PS", "P"):
            raise ValueError("pols placeholder bound to %s" % (t,))
        grouped[i] = t
    opnds = [r for r in grouped if r[0] != "OFF"]
    if cls == "Goldilocks":
        op = {"add": "add", "sub": "sub", "mul": "mul", "mult": "mul", "copy": "copy"}[fn]
        da = db = 1
        dd = 1
    else:
        op, da, db = dims_of(fn)
        op = "mul" if op == "mult" else op
        dd = 3
    n = 2 if op == "copy" else 3
    if len(opnds) != n:
        raise ValueError("%d operands for %s: %s" % (len(opnds), stmt[:120], opnds))

    def with_dim(o, d):
        if o[0] in ("P", "PS"):
            return (o[0], d) + tuple(o[1:])
        return o

    if op == "copy":
        ops.append(("copy", with_dim(opnds[0], dd), with_dim(opnds[1], da if cls == "Goldilocks3" else 1), None))
    else:
        ops.append((op, with_dim(opnds[0], dd), with_dim(opnds[1], da), with_dim(opnds[2], db)))
    return ops


def parse_case(txt):
    """micro-operations and argument count of one opcode"""
    base = 0
    offsets = {}
    ops = []
    stmts = [s.strip() for s in txt.replace("{", ";").replace("}", ";").split(";")]
    q_store = "params.q_2ns" in txt
    if q_store:
        # opcode 69: q_2ns[(i+j)*3] = zhInv(i+j) * tmp3[args[i_args]] (per lane)
        m = re.search(r"tmp3\[" + A + r"\]", txt)
        ops.append(("qout", ("Q",), ("ZI",), ("T3", int(m.group(1) or 0))))
        n = re.search(r"i_args \+= (\d+)", txt)
        return ops, int(n.group(1))
    for s in stmts:
        if not s:
            continue
        m = re.fullmatch(r"i_args \+= (\d+)", s)
        if m:
            base += int(m.group(1))
            continue
        if s.startswith("for (uint64_t j") or s.startswith("j < AVX") or s.startswith("++j"):
            continue
        m = re.fullmatch(r"offsets(\d)\[j\] = (.*)", s, re.S)
        if m:
            offsets[int(m.group(1))] = parse_offsets(m.group(2), base)
            continue
        if s.startswith("Goldilocks"):
            ops += statement_ops(s, base, offsets)
            continue
        raise ValueError("unparsed statement %r" % s[:160])
    return ops, base


def extract(ref=REF):
    isa = {}
    for p in PARSERS:
        with open(os.path.join(ref, "zkevm.chelpers.%s.parser.cpp" % p)) as f:
            text = f.read()
        body = function_body(text, "%s_parser_first_avx" % p)
        table = {}
        for opc, txt in sorted(cases(body).items()):
            ops, nargs = parse_case(txt)
            table[opc] = {"nargs": nargs, "ops": ops}
        isa[p] = table
    return isa


def header_sizes(ref=REF):
    """NOPS_/NARGS_/NTEMP1_/NTEMP3_ of each .parser.hpp"""
    out = {}
    for p in PARSERS:
        with open(os.path.join(ref, "zkevm.chelpers.%s.parser.hpp" % p)) as f:
            head = f.read(400)
        out[p] = {k: int(v) for k, v in re.findall(r"#define (\w+)_ (\d+)", head)}
    return out


def load_bytecode(step, ref=REF):
    """(ops, args) arrays of one parser's bytecode, read at test time only."""
    import numpy as np
    with open(os.path.join(ref, "zkevm.chelpers.%s.parser.hpp" % step)) as f:
        text = f.read()
    arrs = re.findall(r"uint64_t (\w+)\[\w+\]\s*=\s*\{([^}]*)\}", text)
    got = {}
    for name, body in arrs:
        got[name] = np.array([int(x.strip().rstrip("ULul")) for x in body.replace("\n", " ").split(",") if x.strip()], dtype=np.uint64)
    ops = [v for k, v in got.items() if k.startswith("op")][0]
    args = [v for k, v in got.items() if k.startswith("args")][0]
    return ops, args


# ---------------------------------------------------------------- C table emission
KIND = {"T1": 1, "T3": 2, "P": 3, "PS": 4, "K": 5, "KS": 6, "KL": 7, "L": 8, "C": 9, "CL": 10, "U": 11, "E": 12,
        "EL": 13, "X": 14, "ZI": 15, "XDIV": 16, "XDIVW": 17, "Q": 18, "F": 19, "A": 20}
OPS = {"add": 0, "sub": 1, "mul": 2, "copy": 3, "qout": 4}


def enc_operand(o):
    """-> (kind, dim, f0, f1, f2, f3): f = argument indices or literals, -1 unused"""
    if o is None:
        return (0, 0, -1, -1, -1, -1)
    k = o[0]
    if k in ("P", "PS"):
        d = o[1]
        f = list(o[2:]) + [-1] * (4 - len(o[2:]))
        return (KIND[k], d, *f)
    dim = {"T1": 1, "T3": 3, "K": 1, "KS": 1, "KL": 1, "L": 1, "C": 3, "CL": 3, "U": 1, "E": 3, "EL": 3, "X": 1,
           "ZI": 3, "XDIV": 3, "XDIVW": 3, "Q": 3, "F": 3, "A": 3}[k]
    f = list(o[1:]) + [-1] * (4 - len(o[1:]))
    return (KIND[k], dim, *f)


def emit_inc(isa, path):
    lines = ["// GENERATED by tools/parser_isa.py from the AVX2 case tables of the reference's",
             "// src/starkpil/zkevm/chelpers/zkevm.chelpers.<step>.parser.cpp (read as text): one row per",
             "// micro-operation {parser, opcode, nargs, op, dst, a, b}; operand = {kind, dim, f0..f3}",
             "// (kinds / fields: tools/parser_isa.py docstring).  Verified against a fresh extraction by",
             "// tests/test_parser_isa.py.  Do not edit."]
    for pi, p in enumerate(PARSERS):
        for opc, e in sorted(isa[p].items()):
            for (op, d, a, b) in e["ops"]:
                enc = [enc_operand(x) for x in (d, a, b)]
                lines.append("{%d, %d, %d, %d, %s}," % (pi, opc, e["nargs"], OPS[op], ", ".join(
                    "{%d, %d, {%s}}" % (t[0], t[1], ", ".join(str(v) for v in t[2:])) for t in enc)))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def to_jsonable(isa):
    return {p: {str(k): {"nargs": v["nargs"], "ops": [[op, d, a, b] for (op, d, a, b) in v["ops"]]}
                for k, v in t.items()} for p, t in isa.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=REF)
    ap.add_argument("--emit-inc")
    ap.add_argument("--json")
    a = ap.parse_args()
    isa = extract(a.reference)
    if a.emit_inc:
        emit_inc(isa, a.emit_inc)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(to_jsonable(isa), f, indent=0)
    for p in PARSERS:
        print(p, len(isa[p]), "opcodes,", sum(len(v["ops"]) for v in isa[p].values()), "micro-ops")


if __name__ == "__main__":
    sys.exit(main())
