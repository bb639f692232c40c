"""StarkInfo JSON -> GPU prover description, and the proof JSON writers, on
the CPU (host/stark_info.cpp, host/zkgpu_fri_proof.hpp through
zkgpu_batch_prover --info / --zkin).

The fork-9 starkinfo is not in the reference tree; zkgpu/starkinfo.py writes
the starkinfo of synthetic instances with every key StarkInfo::load reads
(stark_info.cpp:21-454).  The loader must recover the instance: widths,
evMap, plookup and grand-product contexts, and step code whose ZXP programs
compute the same columns as the instance's own programs (oracle evaluator).
The zkin writer must produce proof2zkinStark's layout byte for byte
(json2file = nlohmann dump(4) + newline).
"""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(os.path.dirname(HERE), "zkevm-prover_amd", "bin", "zkgpu_batch_prover")
P = 0xFFFFFFFF00000001


def driver(*args, check=True):
    if not os.path.exists(DRIVER):
        pytest.fail("zkgpu_batch_prover not built (make -C zkevm-prover_amd)")
    r = subprocess.run([DRIVER, *args], capture_output=True, text=True, timeout=120)
    if check:
        assert r.returncode == 0, r.stderr
    return r


class _Prog:
    def __init__(self, d):
        self.instr = [tuple(i) for i in d["instr"]]
        self.opnd = [tuple(o) for o in d["opnd"]]
        self.n_tmp1, self.n_tmp3 = d["nTmp1"], d["nTmp3"]

    def arrays(self):
        return (np.array(self.instr, np.uint32).reshape(-1, 4), np.array(self.opnd, np.uint32).reshape(-1, 4))


def _eval(oracle, prog, S, sc, dom):
    secs = (ctypes.c_void_p * 12)()
    strides = np.zeros(12, np.uint64)
    for k, a in S.items():
        secs[k] = a.ctypes.data
        strides[k] = a.shape[1]
    ins, opn = prog.arrays()
    ins, opn = np.ascontiguousarray(ins), np.ascontiguousarray(opn)
    p = oracle._p
    oracle.lib().oc_zxp_eval(ctypes.c_void_p(ins.ctypes.data), ins.shape[0], ctypes.c_void_p(opn.ctypes.data),
                             max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ctypes.cast(secs, ctypes.c_void_p),
                             ctypes.c_void_p(strides.ctypes.data), dom, p(sc["challenges"]), p(sc["publics"]),
                             p(sc["evals"]), p(sc["x"]), p(sc["xdiv"]), p(sc["xdivw"]), p(sc["zhinv"]),
                             sc["zhinv"].size)


def _inst(**kw):
    from zkgpu.synthetic import SyntheticStark
    if kw.pop("fork9", False):  # the fork-9 widths, next-row reads and shifted stores (synthetic.py)
        return SyntheticStark.fork9(**kw)
    return SyntheticStark(**kw)


@pytest.mark.parametrize("kw", [dict(n_bits=8, t=4, m=2, n_queries=8), dict(n_bits=7, blowup_bits=2, t=3, m=1,
                                                                             n_lookups=1, q_deg=4, n_queries=6),
                                dict(n_bits=7, t=5, m=3, n_lookups=0, with_step3=False, n_queries=4),
                                dict(fork9=True, n_bits=7, n_queries=4)])
def test_loader_recovers_instance(oracle, tmp_path, kw):
    import zkgpu.starkinfo as zs
    inst = _inst(**kw)
    path = tmp_path / "s.starkinfo.json"
    path.write_text(json.dumps(zs.starkinfo(inst)))
    d = json.loads(driver("--info", str(path)).stdout)
    assert (d["nBits"], d["nBitsExt"], d["nQueries"], d["friSteps"]) == (inst.n_bits, inst.n_bits_ext,
                                                                         inst.n_queries, inst.fri_steps)
    assert (d["nCm1"], d["nCm2"], d["nCm3"], d["nCm4"], d["nTmp"], d["nConst"], d["nPublics"], d["qDeg"]) == \
        (inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4, inst.n_tmp, inst.n_const, inst.n_publics, inst.q_deg)
    assert d["evMap"] == [x for e in inst.evmap for x in e]
    assert d["puCtx"] == [x for e in inst.pu for x in e]
    z = d["zCtx"]
    assert sorted(tuple(z[i:i + 3]) for i in range(0, len(z), 3)) == sorted(inst.z_ctx)
    # every step program computes what the instance's program computes
    rng = np.random.default_rng(3)
    for name, src in zs.PROGRAMS:
        ext = name in ("step42ns", "step52ns")
        dom = 1 << (inst.n_bits_ext if ext else inst.n_bits)
        widths = {0: inst.n_cm1, 1: inst.n_cm2, 2: inst.n_cm3, 3: inst.n_tmp, 4: inst.n_const, 5: inst.n_cm1,
                  6: inst.n_cm2, 7: inst.n_cm3, 8: inst.n_cm4, 9: inst.n_const, 10: 3, 11: 3}
        S0 = {k: rng.integers(0, P, size=(dom, max(w, 1)), dtype=np.uint64) for k, w in widths.items()}
        sc = {"challenges": rng.integers(0, P, 24, dtype=np.uint64),
              "publics": rng.integers(0, P, max(inst.n_publics, 1), dtype=np.uint64),
              "evals": rng.integers(0, P, 3 * len(inst.evmap), dtype=np.uint64),
              "x": rng.integers(0, P, dom, dtype=np.uint64), "zhinv": rng.integers(0, P, 2, dtype=np.uint64),
              "xdiv": rng.integers(0, P, (dom, 3), dtype=np.uint64),
              "xdivw": rng.integers(0, P, (dom, 3), dtype=np.uint64)}
        A = {k: v.copy() for k, v in S0.items()}
        B = {k: v.copy() for k, v in S0.items()}
        _eval(oracle, inst.programs[src], A, sc, dom)
        _eval(oracle, _Prog(d["programs"][name]), B, sc, dom)
        for k in S0:
            assert np.array_equal(A[k], B[k]), (name, k)


def test_zkin_writer_byte_identical(oracle, tmp_path):
    """--zkin on the oracle's proof: batch_proof.zkin.json == proof2zkinStark
    layout dumped as json2file does; batch_proof.proof.json has FRIProof's
    structure and converts to the same zkin."""
    import zkgpu.starkinfo as zs
    from oracle.stark_prover import OracleStark
    inst = _inst(n_bits=8, t=4, m=2, n_queries=8)
    o = OracleStark(inst)
    o.witness()
    proof = o.prove()
    si = tmp_path / "s.starkinfo.json"
    si.write_text(json.dumps(zs.starkinfo(inst)))
    flat = tmp_path / "proof.bin"
    zs.flatten(proof, inst).tofile(flat)
    pub = tmp_path / "publics.json"
    pub.write_text(json.dumps([str(int(v)) for v in o.publics]))
    out = tmp_path / "out"
    driver("--zkin", str(si), str(flat), str(pub), str(out))
    got = (out / "batch_proof.zkin.json").read_text()
    assert got == zs.zkin_text(proof, o.publics, inst.n_cm2, inst.n_cm3)
    full = json.loads((out / "batch_proof.proof.json").read_text())
    assert list(full) == ["root1", "root2", "root3", "root4", "evals", "fri", "publics"]
    fri = full["fri"]
    assert len(fri) == len(inst.fri_steps) + 1
    assert fri[0]["root"] == ["0"] * 4 and len(fri[0]["polQueries"][0]) == 5
    assert fri[1]["root"] == proof["s1_root"]
    assert fri[0]["polQueries"][3][2][0] == proof["s0_vals3"][3]
    assert fri[-1] == proof["finalPol"]


def test_zkin_key_order_matches_golden():
    """the reference's own zkin proofs (tests/golden) have the key order
    proof2zkinStark + publics produces (s0_vals2 absent: no stage-2 columns)"""
    import zkgpu.starkinfo as zs
    g = json.load(open(os.path.join(HERE, "golden", "recursive1.zkin.proof_0.json")))
    n_steps = sum(1 for k in g if k.endswith("_root") and k[1:-5].isdigit()) + 1
    proof = {k: g[k] for k in g if k != "publics"}
    for t in ("2",):
        proof["s0_vals" + t], proof["s0_siblings" + t] = [], []
    z = zs.zkin(proof, [int(v) for v in g["publics"]], 0, 1)
    assert list(z) == list(g)
    assert n_steps == 5


@pytest.mark.parametrize("patch,msg", [
    (lambda j: j["varPolMap"][0].update(section="cm9_n"), "string2section() found invalid string=cm9_n"),
    (lambda j: j["step2prev"]["first"][0]["src"][0].update(type="bogus"), "StepType::setType() found invalid type"),
    (lambda j: j["step42ns"]["first"][0].update(op="div"), "StepOperation::setOperation() found invalid type"),
    (lambda j: j["evMap"][0].update(type="tmp"), "EvMap::setType() found invalid type"),
    (lambda j: j.pop("mapSectionsN"), "missing key \"mapSectionsN\""),
    (lambda j: j["step3prev"]["first"][0]["src"].append({"type": "tree1", "id": 0}), "takes 2 sources"),
])
def test_loader_errors_are_loud(tmp_path, patch, msg):
    import zkgpu.starkinfo as zs
    j = zs.starkinfo(_inst(n_bits=6, t=2, m=1, n_queries=4))
    patch(j)
    path = tmp_path / "bad.starkinfo.json"
    path.write_text(json.dumps(j))
    r = driver("--info", str(path), check=False)
    assert r.returncode == 1 and msg in r.stderr, r.stderr
