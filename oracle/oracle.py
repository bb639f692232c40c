"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes binding of the CPU oracle (oracle/build/liboracle.so).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product (zkevm-prover_amd/) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
P = 0xFFFFFFFF00000001

_lib = None


def build(force=False):
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        u64 = ctypes.c_uint64
        ptr = ctypes.POINTER(ctypes.c_uint64)
        sig = {
            "oc_gl_mul": (u64, [u64, u64]),
            "oc_gl_add": (u64, [u64, u64]),
            "oc_gl_sub": (u64, [u64, u64]),
            "oc_gl_inv": (u64, [u64]),
            "oc_gl_pow": (u64, [u64, u64]),
            "oc_gl_w": (u64, [ctypes.c_uint]),
            "oc_gl3_mul": (None, [ptr, ptr, ptr]),
            "oc_powers3": (None, [ptr, ptr, u64]),
            "oc_gl3_inv": (None, [ptr, ptr]),
            "oc_ntt": (None, [ptr, ptr, u64, u64, ctypes.c_int]),
            "oc_dft_naive": (None, [ptr, ptr, u64, u64, ctypes.c_int]),
            "oc_extend_pol": (None, [ptr, ptr, u64, u64, u64]),
            "oc_poseidon_full": (None, [ptr, ptr]),
            "oc_poseidon_hash": (None, [ptr, ptr]),
            "oc_linear_hash": (None, [ptr, ptr, u64]),
            "oc_merkle_num_elements": (u64, [u64]),
            "oc_merkletree": (None, [ptr, ptr, u64, u64]),
            "oc_merkle_root": (None, [ptr, ptr, u64]),
            "oc_merkle_proof_size": (u64, [u64]),
            "oc_merkle_group_proof": (None, [ptr, ptr, ptr, u64, u64, u64]),
            "oc_merkle_root_from_proof": (None, [ptr, ptr, u64, ptr, u64, u64]),
            "oc_transcript_init": (None, [ctypes.c_void_p]),
            "oc_transcript_put": (None, [ctypes.c_void_p, ptr, u64]),
            "oc_transcript_get_fields1": (u64, [ctypes.c_void_p]),
            "oc_transcript_get_field": (None, [ctypes.c_void_p, ptr]),
            "oc_transcript_get_permutations": (None, [ctypes.c_void_p, ptr, u64, u64]),
            "oc_fri_fold": (None, [ptr, ptr, u64, u64, ptr, u64]),
            "oc_fri_fold_group": (None, [ptr, ptr, u64, u64, u64, ptr, u64]),
            "oc_fri_get_transposed": (None, [ptr, ptr, u64, u64]),
            "oc_batch_inverse3": (None, [ptr, ptr, u64]),
            "oc_rand_u64": (u64, [u64, u64, u64, u64]),
            "oc_rand_cols": (None, [ptr, u64, ctypes.c_void_p, u64, u64, u64, u64]),
            "oc_zxp_eval": (None, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, u64, ptr, ptr, ptr, ptr,
                                   ptr, ptr, ptr, u64]),
            "oc_zxc_eval": (None, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, u64, ptr, ptr, ptr, ptr, ptr, ptr, ptr, u64]),
            "oc_calculate_z": (ctypes.c_int, [ptr, u64, ptr, u64, ptr, u64, u64]),
            "oc_parser_eval": (ctypes.c_int, [ctypes.c_int, ptr, u64, ptr, u64, ctypes.c_uint32, ptr, ptr,
                                              ctypes.c_void_p, ptr, u64, u64, u64, ctypes.c_uint32, ctypes.c_uint32,
                                              ptr, ptr, ptr, ptr, ptr, u64, ptr, ptr, ptr, ptr]),
            "oc_parser_eval_rows": (ctypes.c_int, [ctypes.c_int, ptr, u64, ptr, u64, ctypes.c_uint32, ptr, ptr,
                                                   ctypes.c_void_p, ptr, u64, u64, u64, ctypes.c_uint32,
                                                   ctypes.c_uint32, ptr, ptr, ptr, ptr, ptr, u64, ptr, ptr, ptr, ptr,
                                                   ptr, u64, ptr, u64]),
            "oc_evmap": (None, [ptr, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, u64, ptr,
                                ptr, u64, ctypes.c_uint32]),
            "oc_xdivxsub": (None, [ptr, ptr, ptr, u64, ptr, u64]),
            "oc_powers": (None, [ptr, u64, u64, u64]),
            "oc_h1h2": (u64, [ptr, u64, ptr, u64, ptr, u64, ptr, u64, u64, ctypes.c_uint32]),
            "oc_num_threads": (ctypes.c_int, []),
            "oc_set_num_threads": (None, [ctypes.c_int]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def u64(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint64))


# ---------------------------------------------------------------- field
def gl_mul(a, b): return lib().oc_gl_mul(a, b)
def gl_add(a, b): return lib().oc_gl_add(a, b)
def gl_sub(a, b): return lib().oc_gl_sub(a, b)
def gl_inv(a): return lib().oc_gl_inv(a)
def gl_pow(a, e): return lib().oc_gl_pow(a, e)
def gl_w(n): return lib().oc_gl_w(n)


def gl3_mul(a, b):
    a, b = u64(a), u64(b)
    o = np.zeros(3, np.uint64)
    lib().oc_gl3_mul(_p(o), _p(a), _p(b))
    return o


def gl3_inv(a):
    a = u64(a)
    o = np.zeros(3, np.uint64)
    lib().oc_gl3_inv(_p(o), _p(a))
    return o


def h1h2(f, t):
    """Plookup h1/h2 (calculateH1H2_opt1/opt3): f, t are (n,) or (n, 3).
    Returns (h1, h2), or raises ValueError naming the first f row not in t."""
    f, t = u64(f), u64(t)
    n = t.shape[0]
    dim = 1 if t.ndim == 1 else t.shape[1]
    h1 = np.zeros_like(t)
    h2 = np.zeros_like(t)
    miss = lib().oc_h1h2(_p(h1), dim, _p(h2), dim, _p(f), dim, _p(t), dim, n, dim)
    if miss:
        raise ValueError("Number not included: w=%d" % (miss - 1))
    return h1, h2


# ---------------------------------------------------------------- NTT
def ntt(x, inverse=False):
    """x: (n, ncols) or (n,) uint64 row-major; returns the same shape."""
    x = u64(x)
    n = x.shape[0]
    ncols = 1 if x.ndim == 1 else x.shape[1]
    out = np.empty_like(x)
    lib().oc_ntt(_p(out), _p(x), n, ncols, int(inverse))
    return out


def dft_naive(x, inverse=False):
    x = u64(x)
    n = x.shape[0]
    ncols = 1 if x.ndim == 1 else x.shape[1]
    out = np.empty_like(x)
    lib().oc_dft_naive(_p(out), _p(x), n, ncols, int(inverse))
    return out


def extend_pol(x, n_ext):
    x = u64(x)
    n = x.shape[0]
    ncols = 1 if x.ndim == 1 else x.shape[1]
    shape = (n_ext,) if x.ndim == 1 else (n_ext, ncols)
    out = np.empty(shape, np.uint64)
    lib().oc_extend_pol(_p(out), _p(x), n_ext, n, ncols)
    return out


# ---------------------------------------------------------------- Poseidon
def poseidon_full(x):
    x = u64(x)
    assert x.size == 12
    o = np.zeros(12, np.uint64)
    lib().oc_poseidon_full(_p(o), _p(x))
    return o


def poseidon_hash(x):
    x = u64(x)
    o = np.zeros(4, np.uint64)
    lib().oc_poseidon_hash(_p(o), _p(x))
    return o


def linear_hash(x):
    x = u64(x).reshape(-1)
    o = np.zeros(4, np.uint64)
    lib().oc_linear_hash(_p(o), _p(x) if x.size else _p(np.zeros(1, np.uint64)), x.size)
    return o


# ---------------------------------------------------------------- Merkle
def merkletree(src):
    """src: (nrows, ncols) row-major -> nodes array (getTreeNumElements)."""
    src = u64(src)
    nrows = src.shape[0]
    ncols = src.shape[1] if src.ndim == 2 else 1
    nodes = np.zeros(lib().oc_merkle_num_elements(nrows), np.uint64)
    s = src if src.size else np.zeros(1, np.uint64)
    lib().oc_merkletree(_p(nodes), _p(s), ncols, nrows)
    return nodes


def merkle_root(nodes):
    return nodes[-4:].copy()


def merkle_group_proof(nodes, src, idx):
    src = u64(src)
    nrows, ncols = src.shape[0], (src.shape[1] if src.ndim == 2 else 1)
    nsib = lib().oc_merkle_proof_size(nrows)
    proof = np.zeros(ncols + 4 * nsib, np.uint64)
    s = src if src.size else np.zeros(1, np.uint64)
    lib().oc_merkle_group_proof(_p(proof), _p(nodes), _p(s), ncols, nrows, idx)
    return proof[:ncols], proof[ncols:].reshape(-1, 4)


def merkle_root_from_proof(vals, siblings, idx):
    vals = u64(vals).reshape(-1)
    sib = u64(siblings).reshape(-1)
    root = np.zeros(4, np.uint64)
    v = vals if vals.size else np.zeros(1, np.uint64)
    s = sib if sib.size else np.zeros(1, np.uint64)
    lib().oc_merkle_root_from_proof(_p(root), _p(v), vals.size, _p(s), sib.size // 4, idx)
    return root


# ---------------------------------------------------------------- transcript
class Transcript:
    """Transcript (transcript.cpp:4-87) backed by the C oracle."""

    def __init__(self):
        self._buf = ctypes.create_string_buffer(8 * 24 + 8)
        lib().oc_transcript_init(self._buf)

    def put(self, vals):
        v = u64(vals).reshape(-1)
        if v.size:
            lib().oc_transcript_put(self._buf, _p(v), v.size)

    def get_fields1(self):
        return lib().oc_transcript_get_fields1(self._buf)

    def get_field(self):
        o = np.zeros(3, np.uint64)
        lib().oc_transcript_get_field(self._buf, _p(o))
        return o

    def get_permutations(self, n, nbits):
        o = np.zeros(n, np.uint64)
        lib().oc_transcript_get_permutations(self._buf, _p(o), n, nbits)
        return o


# ---------------------------------------------------------------- FRI
def fri_fold(pol, pol_bits, out_bits, special_x, shift_inv):
    pol = u64(pol).reshape(-1)
    out = np.zeros(3 << out_bits, np.uint64)
    sx = u64(special_x)
    lib().oc_fri_fold(_p(out), _p(pol), pol_bits, out_bits, _p(sx), shift_inv)
    return out


def fri_fold_group(vals, g, pol_bits, special_x, shift_inv):
    vals = u64(vals).reshape(-1)
    out = np.zeros(3, np.uint64)
    sx = u64(special_x)
    lib().oc_fri_fold_group(_p(out), _p(vals), vals.size // 3, g, pol_bits, _p(sx), shift_inv)
    return out


def fri_get_transposed(pol, transpose_bits):
    pol = u64(pol).reshape(-1)
    aux = np.zeros_like(pol)
    lib().oc_fri_get_transposed(_p(aux), _p(pol), pol.size // 3, transpose_bits)
    return aux


def batch_inverse3(x):
    x = u64(x).reshape(-1)
    o = np.zeros_like(x)
    lib().oc_batch_inverse3(_p(o), _p(x), x.size // 3)
    return o


def parser_eval(parser, ops, args, sections, cpols, dom, native_dom, n_tmp1, n_tmp3, challenges, publics, evals, x,
                zhinv, xdiv=None, xdivw=None, q=None, f=None):
    """oracle/parser.c: the reference's AVX2 bytecode case tables, one row at a
    time.  sections: [(offset, stride, row-major uint64 array (dom x stride))]
    of the memory map; outputs are written in place.  Returns the status."""
    ops = np.ascontiguousarray(ops, np.uint64)
    args = np.ascontiguousarray(args, np.uint64)
    off = np.array([s[0] for s in sections], np.uint64)
    stride = np.array([s[1] for s in sections], np.uint64)
    ptrs = (ctypes.c_void_p * len(sections))(*[s[2].ctypes.data for s in sections])
    return lib().oc_parser_eval(parser, _p(ops), ops.size, _p(args), args.size, len(sections), _p(off), _p(stride),
                                ctypes.cast(ptrs, ctypes.c_void_p), _p(cpols), cpols.shape[1], dom, native_dom,
                                n_tmp1, n_tmp3, _p(challenges), _p(publics), _p(evals), _p(x), _p(zhinv), zhinv.size,
                                *[_p(a) if a is not None else None for a in (xdiv, xdivw, q, f)])


def parser_eval_rows(parser, ops, args, sections, cpols, dom, native_dom, n_tmp1, n_tmp3, challenges, publics, evals,
                     x, zhinv, rows, rmap, xdiv=None, xdivw=None, q=None, f=None):
    """oracle/parser.c oc_parser_eval_rows: the interpreter on the rows `rows`
    of a dom-row domain; every row-indexed array (sections, cpols, x, xdiv,
    xdivw, q, f) holds only the rows of `rmap` (sorted ascending), in that
    order.  Returns the status."""
    ops = np.ascontiguousarray(ops, np.uint64)
    args = np.ascontiguousarray(args, np.uint64)
    rows = np.ascontiguousarray(rows, np.uint64)
    rmap = np.ascontiguousarray(rmap, np.uint64)
    off = np.array([s[0] for s in sections], np.uint64)
    stride = np.array([s[1] for s in sections], np.uint64)
    for s in sections:
        assert s[2].shape == (rmap.size, s[1]) and s[2].flags.c_contiguous
    ptrs = (ctypes.c_void_p * len(sections))(*[s[2].ctypes.data for s in sections])
    return lib().oc_parser_eval_rows(parser, _p(ops), ops.size, _p(args), args.size, len(sections), _p(off),
                                     _p(stride), ctypes.cast(ptrs, ctypes.c_void_p), _p(cpols), cpols.shape[1], dom,
                                     native_dom, n_tmp1, n_tmp3, _p(challenges), _p(publics), _p(evals), _p(x),
                                     _p(zhinv), zhinv.size,
                                     *[_p(a) if a is not None else None for a in (xdiv, xdivw, q, f)],
                                     _p(rows), rows.size, _p(rmap), rmap.size)
