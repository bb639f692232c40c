"""The reference's input files for a STARK instance, from a synthetic one.

zkgpu_batch_prover (host/batch_prover.cpp) proves from the files the
reference's batch prover reads (config.cpp:231-242): <circuit>.starkinfo.json
(StarkInfo::load, stark_info.cpp:21-454), the constant polynomials, the
constant tree and the committed trace.  The fork-9 files are not in the
reference tree, so the tests write them for a zkgpu.synthetic.SyntheticStark:

  starkinfo(inst)      the starkinfo JSON: starkStruct, the memory map
                       (mapSectionsN / mapDeg / mapOffsets / mapSections /
                       N1 / N3), varPolMap with cm_n / cm_2ns / qs / exps_n /
                       exp2pol, evMap, puCtx / peCtx / ciCtx and the step code
                       (step2prev, step3prev, step3, step42ns, step52ns) as
                       StepOperation lists (stark_info.hpp:148-260)
  write_inputs(...)    those files + a config JSON for the driver
  zkin_text(...)       the zkin JSON the driver must write, as text

Committed polynomial order (cm_n / cm_2ns): the cm1 columns, then h1 / h2 of
each plookup, then the Z of each plookup and of each permutation context --
the positions transposeH1H2Columns / transposeZColumns read (starks.cpp:14,
406-520) -- then the other stage-2/3 columns and the quotient pieces.
"""
import json
import os

import numpy as np

from . import synthetic as sy

P = 0xFFFFFFFF00000001
# eSection names (stark_info.hpp:42-55)
SECTIONS = ["cm1_n", "cm1_2ns", "cm2_n", "cm2_2ns", "cm3_n", "cm3_2ns", "cm4_n", "cm4_2ns", "tmpExp_n", "q_2ns",
            "f_2ns"]
ZXP_SEC_NAME = {sy.SEC_CM1_N: "cm1_n", sy.SEC_CM2_N: "cm2_n", sy.SEC_CM3_N: "cm3_n", sy.SEC_TMP_N: "tmpExp_n",
                sy.SEC_CM1_2NS: "cm1_2ns", sy.SEC_CM2_2NS: "cm2_2ns", sy.SEC_CM3_2NS: "cm3_2ns",
                sy.SEC_CM4_2NS: "cm4_2ns", sy.SEC_Q_2NS: "q_2ns", sy.SEC_F_2NS: "f_2ns"}
N_OF = {"cm1_2ns": "cm1_n", "cm2_2ns": "cm2_n", "cm3_2ns": "cm3_n", "cm4_2ns": "cm4_n"}
OPS = {sy.ADD: "add", sy.SUB: "sub", sy.MUL: "mul", sy.COPY: "copy"}
PROGRAMS = [("step2prev", "step2"), ("step3prev", "step3prev"), ("step3", "step3"), ("step42ns", "step42ns"),
            ("step52ns", "step52ns")]


class _Builder:
    def __init__(self, inst):
        self.inst = inst
        self.var = []       # varPolMap entries
        self.vidx = {}
        self.cm_n, self.cm_2ns = [], []
        self.cidx = {}      # (n section, col, dim) -> committed index
        self.exps = []      # exps_n: polId per expression
        self.eidx = {}      # (col, dim) -> expression id

    def pol(self, section, col, dim):
        key = (section, col, dim)
        if key not in self.vidx:
            self.vidx[key] = len(self.var)
            self.var.append({"section": section, "sectionPos": col, "dim": dim})
        return self.vidx[key]

    def committed(self, nsec, col, dim):
        key = (nsec, col, dim)
        if key not in self.cidx:
            self.cidx[key] = len(self.cm_n)
            esec = {v: k for k, v in N_OF.items()}[nsec]
            self.cm_n.append(self.pol(nsec, col, dim))
            self.cm_2ns.append(self.pol(esec, col, dim))
        return self.cidx[key]

    def exp(self, col, dim):
        key = (col, dim)
        if key not in self.eidx:
            self.eidx[key] = len(self.exps)
            self.exps.append(self.pol("tmpExp_n", col, dim))
        return self.eidx[key]


def _committed_order(b, inst):
    for c in range(inst.n_cm1):
        b.committed("cm1_n", c, 1)
    for lk in inst.lookups:
        b.committed("cm2_n", lk["h1"], lk["dim"])
        b.committed("cm2_n", lk["h2"], lk["dim"])
    for lk in inst.lookups:
        b.committed("cm3_n", lk["z"], 3)
    for j in range(inst.m):
        b.committed("cm3_n", inst.z_ctx[j][2], 3)
    for j in range(inst.m):
        b.committed("cm2_n", 3 * j, 3)
    if inst.with_step3:
        b.committed("cm3_n", inst.cm3_w, 3)
    for p in range(inst.q_deg):
        b.committed("cm4_n", 3 * p, 3)


def _operand(b, inst, prog, k, ext):
    kind, a, bb, c = prog.opnd[k]
    nxt = (1 << inst.blowup_bits) if ext else 1

    def prime(t):
        if c:
            assert c == nxt, "step code has only row and next-row references (shift %d)" % c
            t["prime"] = True
        return t

    if kind in (sy.TMP1, sy.TMP3):
        return {"type": "tmp", "id": a if kind == sy.TMP1 else prog.n_tmp1 + a}
    if kind in (sy.COL, sy.COL3):
        dim = 3 if kind == sy.COL3 else 1
        if a in (sy.SEC_CONST_N, sy.SEC_CONST_2NS):
            assert dim == 1
            return prime({"type": "const", "id": bb})
        if a == sy.SEC_TMP_N:
            return prime({"type": "exp", "id": b.exp(bb, dim)})
        if a in (sy.SEC_Q_2NS, sy.SEC_F_2NS):
            assert bb == 0 and dim == 3 and not c
            return {"type": "q" if a == sy.SEC_Q_2NS else "f", "id": 0}
        name = ZXP_SEC_NAME[a]
        return prime({"type": "cm", "id": b.committed(N_OF.get(name, name), bb, dim)})
    if kind == sy.LIT:
        return {"type": "number", "value": str(a | (bb << 32))}
    if kind == sy.PUB:
        return {"type": "public", "id": a}
    if kind == sy.CHAL:
        return {"type": "challenge", "id": a}
    if kind == sy.EVAL:
        return {"type": "eval", "id": a}
    return {"type": {sy.X: "x", sy.XDIV: "xDivXSubXi", sy.XDIVW: "xDivXSubWXi", sy.ZI: "Zi"}[kind]}


def _step(b, inst, prog, ext):
    code = []
    for op, d, x, y in prog.instr:
        src = [_operand(b, inst, prog, x, ext)]
        if op != sy.COPY:
            src.append(_operand(b, inst, prog, y, ext))
        code.append({"op": OPS[op], "dest": _operand(b, inst, prog, d, ext), "src": src})
    return {"tmpUsed": prog.n_tmp1 + prog.n_tmp3, "first": code, "i": [], "last": []}


def starkinfo(inst):
    """The starkinfo JSON (dict) of a SyntheticStark."""
    b = _Builder(inst)
    _committed_order(b, inst)
    steps = {name: _step(b, inst, inst.programs[src], name in ("step42ns", "step52ns")) for name, src in PROGRAMS}
    # contexts (stark_info.cpp:149-186): expressions by id, exp2pol maps them to tmpExp_n
    pu = [{"tExpId": b.exp(lk["t"], lk["dim"]), "fExpId": b.exp(lk["f"], lk["dim"]), "h1Id": 0, "h2Id": 0, "zId": 0,
           "c1Id": 0, "numId": b.exp(lk["num"], 3), "denId": b.exp(lk["den"], 3), "c2Id": 0} for lk in inst.lookups]
    pe = [{"tExpId": 0, "fExpId": 0, "zId": 0, "c1Id": 0, "numId": b.exp(inst.z_ctx[j][0], 3),
           "denId": b.exp(inst.z_ctx[j][1], 3), "c2Id": 0} for j in range(inst.m)]
    qs = [b.pol("cm4_2ns", 3 * p, 3) for p in range(inst.q_deg)]
    ev = []
    for sec, col, dim, prime in inst.evmap:
        if sec == sy.SEC_CONST_2NS:
            ev.append({"type": "const", "id": col, "prime": bool(prime)})
        elif sec == sy.SEC_CM4_2NS:
            ev.append({"type": "q", "id": col // 3, "prime": bool(prime)})
        else:
            ev.append({"type": "cm", "id": b.committed(N_OF[ZXP_SEC_NAME[sec]], col, dim), "prime": bool(prime)})
    N, NE = 1 << inst.n_bits, 1 << inst.n_bits_ext
    width = {"cm1_n": inst.n_cm1, "cm1_2ns": inst.n_cm1, "cm2_n": inst.n_cm2, "cm2_2ns": inst.n_cm2,
             "cm3_n": inst.n_cm3, "cm3_2ns": inst.n_cm3, "cm4_n": inst.n_cm4, "cm4_2ns": inst.n_cm4,
             "tmpExp_n": inst.n_tmp, "q_2ns": 3, "f_2ns": 3}
    deg = {s: (NE if s.endswith("2ns") else N) for s in SECTIONS}
    offs, o = {}, 0
    for s in SECTIONS:
        offs[s] = o
        o += width[s] * deg[s]
    sec_pols = {s: [i for i, v in enumerate(b.var) if v["section"] == s] for s in SECTIONS}
    n_dim = lambda s, d: sum(1 for i in sec_pols[s] if b.var[i]["dim"] == d)  # noqa: E731
    stage = lambda s: sum(1 for k in b.cm_n if b.var[k]["section"] == s)  # noqa: E731
    return {
        "varPolMap": b.var,
        "qs": qs,
        "cm_n": b.cm_n,
        "cm_2ns": b.cm_2ns,
        "peCtx": pe,
        "puCtx": pu,
        "ciCtx": [],
        "evMap": ev,
        "starkStruct": {"nBits": inst.n_bits, "nBitsExt": inst.n_bits_ext, "nQueries": inst.n_queries,
                        "verificationHashType": "GL", "steps": [{"nBits": s} for s in inst.fri_steps]},
        "nConstants": inst.n_const,
        "nPublics": inst.n_publics,
        "nCm1": stage("cm1_n"),
        "nCm2": stage("cm2_n"),
        "nCm3": stage("cm3_n"),
        "nCm4": stage("cm4_n"),
        "qDeg": inst.q_deg,
        "qDim": 3,
        "friExpId": 0,
        "nExps": len(b.exps),
        "mapTotalN": o,
        "mapDeg": deg,
        "mapOffsets": offs,
        "mapSections": sec_pols,
        "mapSectionsN": width,
        "mapSectionsN1": {s: n_dim(s, 1) for s in SECTIONS},
        "mapSectionsN3": {s: n_dim(s, 3) for s in SECTIONS},
        **steps,
        "exps_n": b.exps,
        "q_2ns": [None] * len(b.exps),
        "cm4_n": [b.pol("cm4_n", 3 * p, 3) for p in range(inst.q_deg)],
        "cm4_2ns": qs,
        "tmpExp_n": b.exps,
        "exp2pol": {str(e): pid for e, pid in enumerate(b.exps)},
    }


def write_inputs(d, inst, const_rows, const_2ns_rows, const_nodes, cm1_rows, publics):
    """starkinfo + const + const tree + commit + publics files and the driver's
    config (config.cpp key names) under directory d; returns the config path."""
    os.makedirs(d, exist_ok=True)
    si = os.path.join(d, "zkevm.starkinfo.json")
    with open(si, "w") as f:
        json.dump(starkinfo(inst), f, indent=1)
    const = os.path.join(d, "zkevm.const")
    np.ascontiguousarray(const_rows, dtype=np.uint64).tofile(const)
    # const tree: MerkleTreeGL image = [width, height] header, the LDE rows, the nodes (root last)
    tree = os.path.join(d, "zkevm.consttree")
    NE = const_2ns_rows.shape[0]
    np.concatenate([np.array([const_2ns_rows.shape[1], NE], np.uint64),
                    np.ascontiguousarray(const_2ns_rows, dtype=np.uint64).reshape(-1),
                    np.asarray(const_nodes, dtype=np.uint64).reshape(-1)]).tofile(tree)
    cm = os.path.join(d, "zkevm.commit")
    np.ascontiguousarray(cm1_rows, dtype=np.uint64).tofile(cm)
    pub = os.path.join(d, "publics.json")
    with open(pub, "w") as f:
        json.dump([str(int(v) % P) for v in publics], f)
    cfg = {"zkevmStarkInfo": si, "zkevmConstPols": const, "zkevmConstantsTree": tree, "zkevmCmPols": cm,
           "zkgpuPublics": pub, "outputPath": os.path.join(d, "out")}
    path = os.path.join(d, "config.json")
    with open(path, "w") as f:
        json.dump(cfg, f, indent=4)
    return path


def zkin(proof, publics, n_cm2, n_cm3):
    """proof2zkinStark (fri/proof2zkinStark.cpp:8-82) of an oracle proof dict
    (zkin-layout keys), s0_vals2/3 dropped for empty stages, + publics."""
    keys = ["root1", "root2", "root3", "root4", "evals"]
    i = 1
    while "s%d_root" % i in proof:
        keys += ["s%d_root" % i, "s%d_vals" % i, "s%d_siblings" % i]
        i += 1
    tags = ["1"] + (["2"] if n_cm2 else []) + (["3"] if n_cm3 else []) + ["4", "C"]
    keys += ["s0_vals" + t for t in tags] + ["s0_siblings" + t for t in tags] + ["finalPol"]
    out = {k: proof[k] for k in keys}
    out["publics"] = [str(int(v) % P) for v in publics]
    return out


def zkin_text(proof, publics, n_cm2, n_cm3):
    """the driver's batch_proof.zkin.json, byte for byte (json2file: dump(4) + newline)"""
    return json.dumps(zkin(proof, publics, n_cm2, n_cm3), indent=4) + "\n"


def flatten(proof, inst):
    """an oracle proof dict -> the flat u64 layout of include/zkgpu_stark.h"""
    out = []

    def put(v):
        out.extend(int(x) for x in np.asarray(v, dtype=object).reshape(-1))

    for k in ("root1", "root2", "root3", "root4", "evals"):
        put(proof[k])
    for si in range(1, len(inst.fri_steps)):
        for k in ("root", "vals", "siblings"):
            put(proof["s%d_%s" % (si, k)])
    for t in ("1", "2", "3", "4", "C"):
        put(proof["s0_vals" + t])
    for t in ("1", "2", "3", "4", "C"):
        put(proof["s0_siblings" + t])
    put(proof["finalPol"])
    return np.array(out, dtype=np.uint64)
