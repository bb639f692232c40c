"""oracle/parser.c oc_parser_eval_rows (the interpreter on sampled rows of a
domain too large for the host, tests/test_gpu_full_parity.py) == the
whole-domain interpreter on the same inputs, wrap-around rows included."""
import numpy as np
import pytest

P = 0xFFFFFFFF00000001


def _rand(rng, shape):
    return rng.integers(0, P, size=shape, dtype=np.uint64)


def sample_rows(dom, rng, n_random=64, shifts=(1, 2, 3, 4)):
    """the rows a full-size check samples: the first and last rows (the
    (i + s) mod N wrap), both sides of every power-of-two boundary >= 2^8
    (workgroup / launch chunking), random rows; and rmap = those rows plus
    every row a shifted access of theirs reaches"""
    rows = {0, 1, 2, dom - 3, dom - 2, dom - 1}
    k = 256
    while k < dom:
        rows |= {k - 1, k, k + 1}
        k *= 2
    rows |= {int(r) for r in rng.integers(0, dom, n_random)}
    rows = np.array(sorted(rows), np.uint64)
    rmap = sorted({int(r) for r in rows} | {(int(r) + s) % dom for r in rows for s in shifts})
    return rows, np.array(rmap, np.uint64)


@pytest.mark.parametrize("name", ["step42ns", "step52ns"])
def test_rows_equal_whole_domain(oracle, name):
    import zkgpu.synthetic_bytecode as sb
    shape = sb.load_shape()
    pid = sb.PARSERS.index(name)
    ops, args = sb.generate(name, seed=1, scale=0.25)
    secs = sb.sections(shape)
    dom = 1 << 11
    rng = np.random.default_rng(11)
    S = {sec: _rand(rng, (dom, w)) for sec, _, w in secs if sec >= 5}
    const = _rand(rng, (dom, shape["n_const"]))
    chal, pub, evals = _rand(rng, (8, 3)), _rand(rng, 48), _rand(rng, (2048, 3))
    xdiv, xdivw = _rand(rng, (dom, 3)), _rand(rng, (dom, 3))
    x = np.zeros(dom, np.uint64)
    oracle.lib().oc_powers(oracle._p(x), 7, oracle.gl_w(11), dom)
    zh = np.array([pow((pow(7, dom >> 1, P) * pow(P - 1, i, P) - 1) % P, P - 2, P) for i in range(2)], np.uint64)
    off = {sec: o for sec, o, _ in secs}
    sh = shape["programs"][name]
    nt1, nt3 = max(sh["ntemp1"], 8), max(sh["ntemp3"], 4)
    out = "q" if name == "step42ns" else "f"
    full = np.zeros((dom, 3), np.uint64)
    rc = oracle.parser_eval(pid, ops, args, [(off[s], a.shape[1], a) for s, a in S.items()], const, dom,
                            1 << shape["n_bits_ext"], nt1, nt3, chal, pub, evals, x, zh, xdiv, xdivw, **{out: full})
    assert rc == 0 and full.any()
    rows, rmap = sample_rows(dom, rng)
    idx = np.searchsorted(rmap, rows)
    part = np.zeros((rmap.size, 3), np.uint64)
    rc = oracle.parser_eval_rows(pid, ops, args,
                                 [(off[s], a.shape[1], np.ascontiguousarray(a[rmap])) for s, a in S.items()],
                                 np.ascontiguousarray(const[rmap]), dom, 1 << shape["n_bits_ext"], nt1, nt3, chal, pub,
                                 evals, np.ascontiguousarray(x[rmap]), zh, rows, rmap,
                                 np.ascontiguousarray(xdiv[rmap]), np.ascontiguousarray(xdivw[rmap]), **{out: part})
    assert rc == 0
    assert np.array_equal(part[idx], full[rows.astype(np.int64)])


def test_rows_missing_row_is_reported(oracle):
    """a shifted access to a row the caller did not provide: status -5"""
    import zkgpu.synthetic_bytecode as sb
    shape = sb.load_shape()
    ops, args = sb.generate("step42ns", seed=1, scale=0.25)
    secs = sb.sections(shape)
    dom = 1 << 10
    rng = np.random.default_rng(3)
    rows = np.array([5, dom - 1], np.uint64)
    rmap = rows.copy()  # without the next rows the program reads
    S = [(o, w, _rand(rng, (rmap.size, w))) for sec, o, w in secs if sec >= 5]
    q = np.zeros((rmap.size, 3), np.uint64)
    rc = oracle.parser_eval_rows(3, ops, args, S, _rand(rng, (rmap.size, shape["n_const"])), dom,
                                 1 << shape["n_bits_ext"], 1196, 175, _rand(rng, (8, 3)), _rand(rng, 48),
                                 _rand(rng, (4, 3)), _rand(rng, rmap.size), np.ones(2, np.uint64), rows, rmap, q=q)
    assert rc == -5
