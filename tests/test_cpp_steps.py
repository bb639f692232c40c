"""The Steps boundary as the reference calls it: tests/cpp/steps_check.cpp
instantiates zkgpu::StepsGPU<Steps, StepsParams> (host/zkgpu_steps.hpp) against
stand-ins with steps.hpp:4-58's exact signatures and calls it through a Steps&
like Starks::genProof (starks.cpp:73,155,193,241,371).  The outputs it writes
equal the oracle's case-table interpreter (oracle/parser.c) on the same
zkEVM-shaped program and memory map (zkgpu/synthetic_bytecode.py)."""
import copy
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "steps_check")
P = 0xFFFFFFFF00000001
MAGIC = 0x5354455053


def build_steps_check():
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    subprocess.check_call([
        "g++", "-O2", "-std=c++17", "-Wall", "-o", BIN, os.path.join(ROOT, "tests/cpp/steps_check.cpp"),
        "-L" + os.path.join(ROOT, "zkevm-prover_amd/lib"), "-lzkgpu",
        "-Wl,-rpath,$ORIGIN/../zkevm-prover_amd/lib"])
    return BIN


def test_steps_check_compiles():
    """StepsGPU overrides every pure-virtual and whole-domain member of the
    reference's Steps (an abstract leftover would not instantiate)"""
    import zkgpu
    if not os.path.exists(zkgpu.LIB_PATH):
        zkgpu.build()
    assert os.path.exists(build_steps_check())


def _case(name, n_bits, seed):
    """a compact memory map (the program's domain's sections back to back),
    the program, random sections / constants / challenges"""
    import zkgpu.synthetic_bytecode as sb
    shape = copy.deepcopy(sb.load_shape())
    shape["n_bits"], shape["n_bits_ext"] = n_bits, n_bits + 1
    pid = sb.PARSERS.index(name)
    ext = pid >= 3
    dom = 1 << (n_bits + 1 if ext else n_bits)
    base = 0
    for m in shape["map"]:
        if (m["zxp_section"] >= 5) == ext:
            m["offset"] = base
            base += dom * m["width"]
        else:
            m["offset"] = 1 << 40
    ops, args = sb.generate(name, seed=seed, shape=shape)
    secs = sb.sections(shape)
    rng = np.random.default_rng(seed)
    c = dict(name=name, pid=pid, ext=ext, dom=dom, shape=shape, ops=ops, args=args, secs=secs,
             pols=rng.integers(0, P, base, dtype=np.uint64),
             const=rng.integers(0, P, (dom, shape["n_const"]), dtype=np.uint64),
             chal=rng.integers(0, P, (8, 3), dtype=np.uint64), pub=rng.integers(0, P, 48, dtype=np.uint64),
             evals=rng.integers(0, P, (2048 if name == "step52ns" else 4, 3), dtype=np.uint64))
    c["xdiv"] = rng.integers(0, P, (dom, 3), dtype=np.uint64) if name == "step52ns" else None
    c["xdivw"] = rng.integers(0, P, (dom, 3), dtype=np.uint64) if name == "step52ns" else None
    return c


def _write_input(path, c):
    sh = c["shape"]
    hdr = [MAGIC, c["pid"], sh["n_bits"], sh["n_bits_ext"], sh["n_const"], c["pub"].size, len(c["ops"]),
           len(c["args"]), len(c["secs"]), c["pols"].size, c["dom"], c["evals"].shape[0], int(c["xdiv"] is not None)]
    parts = [np.array(hdr, np.uint64), np.asarray(c["ops"], np.uint64), np.asarray(c["args"], np.uint64),
             np.array([v for s in c["secs"] for v in s], np.uint64), c["pols"], c["const"].reshape(-1),
             c["chal"].reshape(-1), c["pub"], c["evals"].reshape(-1)]
    if c["xdiv"] is not None:
        parts += [c["xdiv"].reshape(-1), c["xdivw"].reshape(-1)]
    with open(path, "wb") as f:
        for a in parts:
            f.write(np.ascontiguousarray(a, np.uint64).tobytes())


def _oracle(oracle, c):
    dom, sh = c["dom"], c["shape"]
    x = np.zeros(dom, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), 7 if c["ext"] else 1, oracle.gl_w(int(dom).bit_length() - 1), dom)
    zh = np.array([pow((pow(7, dom >> 1, P) * pow(P - 1, i, P) - 1) % P, P - 2, P) for i in range(2)], np.uint64)
    pols = c["pols"].copy()
    views = [(o, w, pols[o:o + dom * w].reshape(dom, w)) for s, o, w in c["secs"] if (s >= 5) == c["ext"]]
    q = np.zeros((dom, 3), np.uint64)
    f = np.zeros((dom, 3), np.uint64)
    st = sh["programs"][c["name"]]
    z3 = np.zeros((dom, 3), np.uint64)
    rc = oracle.parser_eval(c["pid"], c["ops"], c["args"], views, c["const"], dom, dom, max(st["ntemp1"], 8),
                            max(st["ntemp3"], 4), c["chal"], c["pub"], c["evals"], x, zh,
                            c["xdiv"] if c["xdiv"] is not None else z3, c["xdivw"] if c["xdivw"] is not None else z3,
                            q=q, f=f)
    assert rc == 0
    return pols, q, f


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_bits", [("step42ns", 12), ("step3", 12), ("step52ns", 12), ("step2prev", 12)])
def test_steps_gpu_through_reference_interface(oracle, tmp_path, name, n_bits):
    if not os.path.exists(BIN):
        build_steps_check()
    c = _case(name, n_bits, seed=11)
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    _write_input(inp, c)
    r = subprocess.run([BIN, str(inp), str(out)], capture_output=True, text=True, timeout=240)
    print(r.stdout)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
    got = np.fromfile(out, np.uint64)
    dom, n = c["dom"], c["pols"].size
    pols, q, f = got[:n], got[n:n + 3 * dom].reshape(dom, 3), got[n + 3 * dom:].reshape(dom, 3)
    rp, rq, rf = _oracle(oracle, c)
    assert np.array_equal(pols, rp)
    assert np.array_equal(q, rq)
    assert np.array_equal(f, rf)
    if name == "step42ns":
        assert rq.any()
    elif name == "step52ns":
        assert rf.any()
    else:
        assert not np.array_equal(rp, c["pols"])
