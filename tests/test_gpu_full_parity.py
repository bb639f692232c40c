"""Parity at the benchmarked sizes (VERDICT r4 "next" item 2).

* The config-4 proof bench.py times (bench.stark_instance(23, ...): 2^23-row
  trace, 100/26/27/6 committed columns, 128 queries) == the oracle's proof of
  the same instance, field by field: tests/golden/config4_2p23_proof.json,
  written in the build container by tests/golden/make_config4_fixture.py
  (per-field SHA-256 of the canonical JSON, roots / evals / finalPol
  verbatim); likewise the zkEVM-shaped instance at 2^20 rows
  (zkevm_shaped_2p20_proof.json).
* The compiled zkEVM-shaped step42ns (constraint quotient, starks.cpp:241) and
  step52ns (FRI polynomial, starks.cpp:371) kernels at their real 2^24-row
  extended domain -- the segment kernels, carries and scratch columns bench.py
  times -- on ~1,000 sampled rows: the first and last rows (the (i + 2) mod N
  wrap of the next-row reads), both sides of every power-of-two row boundary,
  random rows; each compared with the oracle's case-table interpreter
  evaluating exactly those rows (oracle/parser.c oc_parser_eval_rows, checked
  against the whole-domain interpreter in tests/test_oracle_rows.py).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0xFFFFFFFF00000001
SEC_CONST_2NS, SEC_Q_2NS, SEC_F_2NS = 9, 10, 11


@pytest.mark.parametrize("mode", ["auto", "lean"])
@pytest.mark.parametrize("fixture", ["config4_2p23_proof.json", "zkevm_shaped_2p20_proof.json"])
def test_full_size_proof_equals_oracle_fixture(zkgpu, fixture, mode):
    """config4_2p23: the headline instance at its benchmarked size;
    zkevm_shaped_2p20: the fork-9 widths with the five zkEVM-shaped programs
    (the sharded_one_proof.fork9_zkevm_shaped workload) at the largest size
    whose oracle run fits the build container.  Both under the default plan
    (resident: they fit) and under the lean one (ZKGPU_MEM_LEAN: sections
    sharing one arena by lifetime, cm1 / cm3 extended in place, evmap from the
    extended rows) -- the same proof."""
    import bench
    import torch
    from zkgpu.stark import GpuStark, MEM_AUTO, MEM_LEAN
    from golden.make_config4_fixture import summarize
    torch.cuda.empty_cache()
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", fixture)))
    i = fx["instance"]
    kind = "zkevm" if i.get("kind") == "zkevm" else False
    inst = bench.stark_instance(i["log_n"], i["blowup_bits"], i["ncols"], i["queries"], kind)
    assert [inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4] == i["n_cm"] and inst.n_const == i["n_const"]
    g = GpuStark(inst, mode=MEM_LEAN if mode == "lean" else MEM_AUTO)
    try:
        assert g.memory_mode() == ("lean" if mode == "lean" else "resident")
        g.witness()
        got = summarize(g.prove())
    finally:
        g.close()
    for k, v in fx["small"].items():
        assert got["small"][k] == v, k
    bad = [k for k in fx["fields"] if got["fields"].get(k) != fx["fields"][k]]
    assert not bad, "proof fields differing from the oracle's at 2^%d: %s" % (i["log_n"], bad)
    assert got["digest"] == fx["digest"]


# ---------------------------------------------------------------- zkEVM-shaped programs at 2^24 rows
@pytest.fixture(scope="module")
def full_sections(zkgpu):
    """the fork-9 2ns sections (cm1..cm4 + constants, 1,567 columns) of the
    2^24-row extended domain in HBM (~210 GB), seeded"""
    import torch
    import zkgpu.synthetic_bytecode as sb
    shape = sb.load_shape()
    secs = sb.sections(shape)
    log_dom = shape["n_bits_ext"]
    dom = 1 << log_dom
    g = torch.Generator(device="cuda")
    g.manual_seed(0x24)
    d = {}
    for sec, _, w in secs:
        if sec >= 5:
            d[sec] = (torch.randint(0, 2**63 - 1, (w, dom), dtype=torch.int64, device="cuda", generator=g), dom, w)
    d[SEC_CONST_2NS] = (torch.randint(0, 2**63 - 1, (shape["n_const"], dom), dtype=torch.int64, device="cuda",
                                      generator=g), dom, shape["n_const"])
    yield shape, secs, log_dom, d
    d.clear()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _host_rows(t, idx):
    """rows idx of a device (w, ld) column-major section -> host (len(idx), w)"""
    return np.ascontiguousarray(t[:, idx].cpu().numpy().view(np.uint64).T)


@pytest.mark.parametrize("name", ["step42ns", "step52ns"])
def test_zkevm_shaped_kernels_full_domain_sampled_rows(oracle, zkgpu, full_sections, monkeypatch, name):
    import torch
    import zkgpu.parser as zp
    import zkgpu.synthetic_bytecode as sb
    from test_oracle_rows import sample_rows
    shape, secs, log_dom, dsecs = full_sections
    dom = 1 << log_dom
    monkeypatch.setenv("ZKGPU_ZXP_JIT", "2")
    pid = sb.PARSERS.index(name)
    ops, args = sb.generate(name, seed=1)
    prog = zp.convert(pid, ops, args, secs, shape["n_bits"], shape["n_bits_ext"])
    rng = np.random.default_rng(pid)
    chal, pub, evals = (rng.integers(0, P, s, dtype=np.uint64) for s in ((8, 3), 48, (2048, 3)))
    assert zkgpu.zxp_jit_cached(prog, chal, pub, evals), "compiled kernel not cached: run build()"
    out = torch.zeros((3, dom), dtype=torch.int64, device="cuda")
    d = dict(dsecs)
    xdiv = xdivw = None
    if name == "step42ns":
        d[SEC_Q_2NS] = (out, dom, 3)
    else:
        d[SEC_F_2NS] = (out, dom, 3)
        g = torch.Generator(device="cuda")
        g.manual_seed(0x52)
        xdiv = torch.randint(0, 2**63 - 1, (dom, 3), dtype=torch.int64, device="cuda", generator=g)
        xdivw = torch.randint(0, 2**63 - 1, (dom, 3), dtype=torch.int64, device="cuda", generator=g)
    zkgpu.prof_reset()
    zkgpu.prof_enable(True)
    zkgpu.zxp_eval_dev(prog, d, log_dom, chal, pub, evals, xdiv=xdiv, xdivw=xdivw, extend_bits=1, x_start=7)
    torch.cuda.synchronize()
    zkgpu.prof_enable(False)
    ran = [k for k in zkgpu.prof_kernels() if k.startswith("k_zxp_jit")]
    assert ran, "the compiled kernels did not run"
    if name == "step42ns":
        assert len(ran) > 1, ("the quotient ran as one kernel, not as segments", ran)
    rows, rmap = sample_rows(dom, rng, n_random=900)
    assert rows[-2] == dom - 2 and rows[-1] == dom - 1
    idx = torch.from_numpy(rmap.astype(np.int64)).to("cuda")
    got = np.ascontiguousarray(out[:, idx].cpu().numpy().view(np.uint64).T)
    off = {sec: o for sec, o, _ in secs}
    sections = [(off[sec], w, _host_rows(t, idx)) for sec, (t, _, w) in dsecs.items() if sec != SEC_CONST_2NS]
    const = _host_rows(dsecs[SEC_CONST_2NS][0], idx)
    w = oracle.gl_w(log_dom)
    x = np.array([7 * pow(w, int(r), P) % P for r in rmap], np.uint64)
    zh = np.array([pow((pow(7, dom >> 1, P) * pow(P - 1, i, P) - 1) % P, P - 2, P) for i in range(2)], np.uint64)
    sh = shape["programs"][name]
    ref = np.zeros((rmap.size, 3), np.uint64)
    kw = {"q": ref} if name == "step42ns" else {
        "f": ref, "xdiv": np.ascontiguousarray(xdiv[idx].cpu().numpy().view(np.uint64)),
        "xdivw": np.ascontiguousarray(xdivw[idx].cpu().numpy().view(np.uint64))}
    rc = oracle.parser_eval_rows(pid, ops, args, sections, const, dom, 1 << shape["n_bits_ext"],
                                 max(sh["ntemp1"], 8), max(sh["ntemp3"], 4), chal, pub, evals, x, zh, rows, rmap, **kw)
    assert rc == 0
    k = np.searchsorted(rmap, rows)
    assert ref[k].any()
    bad = [int(r) for r, a, b in zip(rows, got[k], ref[k]) if not np.array_equal(a, b)]
    assert not bad, "%s at 2^%d: %d of %d sampled rows differ, first %s" % (name, log_dom, len(bad), rows.size, bad[:8])
    del out, xdiv, xdivw
    torch.cuda.empty_cache()
