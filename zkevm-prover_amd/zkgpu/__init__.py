"""zkgpu -- Python binding of libzkgpu (the MI355X HIP STARK hot path).

Thin ctypes layer over the C-ABI declared in include/zkgpu.h.  Host-pointer
calls take numpy uint64 arrays (row-major, like the reference); *_dev calls
take device addresses (ints) or torch tensors (int64/uint64 storage,
column-major: column c at base + c*ld elements).

There is no CPU fallback: if lib/libzkgpu.so is missing or no GPU is
present, calls raise ZkgpuError.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
# ZKGPU_LIB_DIR: an alternative build of both libraries (A/B runs of compiler options)
LIB_DIR = os.environ.get("ZKGPU_LIB_DIR") or os.path.join(PKG_ROOT, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libzkgpu.so")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "zkgpu.h")

P = 0xFFFFFFFF00000001


class ZkgpuError(RuntimeError):
    pass


_lib = None

u64 = ctypes.c_uint64
u32 = ctypes.c_uint32
vp = ctypes.c_void_p
pu64 = ctypes.POINTER(ctypes.c_uint64)

_SIGS = {
    "zkgpu_init": (ctypes.c_int, [ctypes.c_int]),
    "zkgpu_release": (None, []),
    "zkgpu_last_error": (ctypes.c_char_p, []),
    "zkgpu_set_stream": (ctypes.c_int, [vp]),
    "zkgpu_synchronize": (ctypes.c_int, []),
    "zkgpu_get_stream": (ctypes.c_void_p, []),
    "zkgpu_abi_version": (ctypes.c_int, []),
    "zkgpu_gl_ntt": (ctypes.c_int, [vp, vp, u64, u64, ctypes.c_int]),
    "zkgpu_gl_extend_pol": (ctypes.c_int, [vp, vp, u64, u64, u64]),
    "zkgpu_gl_ntt_dev": (ctypes.c_int, [vp, u64, vp, u64, u64, u64, ctypes.c_int]),
    "zkgpu_gl_extend_pol_dev": (ctypes.c_int, [vp, u64, vp, u64, u64, u64, u64]),
    "zkgpu_gl_extend_pol_inplace_dev": (ctypes.c_int, [vp, u64, u64, u64]),
    "zkgpu_set_lde_batch_cols": (None, [u64]),
    "zkgpu_gl_merkletree2_dev": (ctypes.c_int, [vp, vp, vp, u64, u64, u64, u64]),
    "zkgpu_rows_to_cols_dev": (ctypes.c_int, [vp, u64, vp, u64, u64]),
    "zkgpu_cols_to_rows_dev": (ctypes.c_int, [vp, vp, u64, u64, u64]),
    "zkgpu_gl_poseidon_full": (ctypes.c_int, [vp, vp]),
    "zkgpu_gl_poseidon_full_host": (ctypes.c_int, [vp, vp]),
    "zkgpu_zxp_eval_block_dev": (ctypes.c_int, [vp, u32, vp, u32, u32, u32, vp, u32, u32, vp, vp, u32, vp, u32, vp,
                                                vp, u32, u64]),
    "zkgpu_gl_poseidon_hash": (ctypes.c_int, [vp, vp]),
    "zkgpu_gl_linear_hash": (ctypes.c_int, [vp, vp, u64]),
    "zkgpu_gl_poseidon_batch_dev": (ctypes.c_int, [vp, vp, u64, ctypes.c_int]),
    "zkgpu_gl_merkle_num_elements": (u64, [u64]),
    "zkgpu_gl_merkletree": (ctypes.c_int, [vp, vp, u64, u64]),
    "zkgpu_const_tree_num_elements": (u64, [u64, u32]),
    "zkgpu_build_const_tree": (ctypes.c_int, [vp, vp, u64, u32, u32]),
    "zkgpu_load_rows_dev": (ctypes.c_int, [vp, u64, vp, u64, u64, u64, ctypes.c_int]),
    "zkgpu_load_rows_stage_bytes": (u64, [u64, u64, u64]),
    "zkgpu_load_rows_async": (ctypes.c_int, [vp, u64, vp, u64, u64, u64, vp, u64, ctypes.POINTER(vp)]),
    "zkgpu_load_wait": (ctypes.c_int, [vp]),
    "zkgpu_gl_merkletree_dev": (ctypes.c_int, [vp, vp, u64, u64, u64]),
    "zkgpu_gl_merkletree_rows_dev": (ctypes.c_int, [vp, vp, u64, u64]),
    "zkgpu_gl_merkle_open_dev": (ctypes.c_int, [vp, vp, vp, vp, u64, u64, u64, vp, u64]),
    "zkgpu_fri_fold_dev": (ctypes.c_int, [vp, vp, u32, u32, vp, u64]),
    "zkgpu_fri_fold_rows_dev": (ctypes.c_int, [vp, vp, u64, u64, u32, u32, vp, u64]),
    "zkgpu_fri_transpose_dev": (ctypes.c_int, [vp, vp, u64, u32]),
    "zkgpu_gl_field_selftest_dev": (ctypes.c_int, [vp, vp, vp, u64, ctypes.c_int]),
    "zkgpu_gl_field_selftest_rb_dev": (ctypes.c_int, [vp, vp, vp, vp, u64, ctypes.c_int, ctypes.c_int]),
    "zkgpu_dev_malloc": (ctypes.c_int, [ctypes.POINTER(vp), u64]),
    "zkgpu_dev_free": (ctypes.c_int, [vp]),
    "zkgpu_memcpy_h2d": (ctypes.c_int, [vp, vp, u64]),
    "zkgpu_memcpy_d2h": (ctypes.c_int, [vp, vp, u64]),
    "zkgpu_memcpy_d2d": (ctypes.c_int, [vp, vp, u64]),
    "zkgpu_memset_dev": (ctypes.c_int, [vp, ctypes.c_int, u64]),
    "zkgpu_rand_cols_dev": (ctypes.c_int, [vp, u64, vp, u32, u64, u64, u64]),
    "zkgpu_rand_cols_rows_dev": (ctypes.c_int, [vp, u64, vp, u32, u64, u64, u32, u64, u64]),
    "zkgpu_copy_rows_dev": (ctypes.c_int, [vp, u64, u64, vp, vp, u64, u64, u32, vp, u32, u64]),
    "zkgpu_device_memory": (ctypes.c_int, [pu64, pu64]),
    "zkgpu_lde_workspace_bytes": (u64, [u64, u64, u64]),
    "zkgpu_zxp_eval_dev": (ctypes.c_int, [vp, u32, vp, u32, u32, u32, vp, u32, vp, vp, u32, vp, u32, vp, vp, u32,
                                          u64]),
    "zkgpu_zxp_compile": (ctypes.c_int, [vp, u32, vp, u32, u32, u32, vp, vp, u32, vp, u32, u32, vp]),
    "zkgpu_zxp_jit_source": (ctypes.c_int, [vp, u32, vp, u32, u32, u32, vp, vp, u32, vp, u32, vp, u64,
                                            ctypes.c_int]),
    "zkgpu_calculate_z_dev": (ctypes.c_int, [vp, u64, vp, u64, vp, u64, u64, ctypes.POINTER(ctypes.c_int)]),
    "zkgpu_calculate_z_block_dev": (ctypes.c_int, [vp, u64, vp, u64, vp, u64, u64, vp, vp]),
    "zkgpu_evmap_dev": (ctypes.c_int, [vp, vp, vp, vp, vp, u32, vp, vp, u64, u64, u32]),
    "zkgpu_xdivxsub_dev": (ctypes.c_int, [vp, vp, vp, u32, u32]),
    "zkgpu_xdivxsub_rows_dev": (ctypes.c_int, [vp, vp, vp, u32, u32, u64, u64]),
    "zkgpu_lagrange_xi_rows_dev": (ctypes.c_int, [vp, vp, u64, vp, u32, u64, u64]),
    "zkgpu_ext_powers_dev": (ctypes.c_int, [vp, u64, vp, u64]),
    "zkgpu_qsplit_dev": (ctypes.c_int, [vp, u64, vp, u64, u64, u32, u64]),
    "zkgpu_qsplit_cols_dev": (ctypes.c_int, [vp, u64, vp, u64, u64, u32, u64, u32, u32]),
    "zkgpu_scale_by_powers_dev": (ctypes.c_int, [vp, u64, u32, u64, u64]),
    "zkgpu_cols3_to_interleaved_dev": (ctypes.c_int, [vp, vp, u64, u64]),
    "zkgpu_h1h2_dev": (ctypes.c_int, [vp, u64, vp, u64, vp, u64, vp, u64, u64, u32, pu64]),
    "zkgpu_h1h2_shard_route": (ctypes.c_int, [vp, u64, vp, vp, vp, u64, vp, u64, u64, u64, u32, u32]),
    "zkgpu_h1h2_shard_owner": (ctypes.c_int, [vp, vp, u64, u32, pu64]),
    "zkgpu_h1h2_shard_counts": (ctypes.c_int, [vp, vp, pu64, vp, vp, u64, u64, u64]),
    "zkgpu_h1h2_shard_deal": (ctypes.c_int, [vp, u64, vp, u64, vp, vp, u64, u32]),
    "zkgpu_h1h2_shard_place": (ctypes.c_int, [vp, u64, vp, u64, vp, u64, u64, u64, u64, u32]),
    "zkgpu_gl_merkle_open_rows_dev": (ctypes.c_int, [vp, vp, vp, vp, u64, u64, vp, u64]),
    "zkgpu_gl_merkle_open_many": (ctypes.c_int, [vp, u32]),
    "zkgpu_calculate_z_many_dev": (ctypes.c_int, [vp, u32, u64, vp]),
    "zkgpu_prof_enable": (ctypes.c_int, [ctypes.c_int]),
    "zkgpu_prof_reset": (ctypes.c_int, []),
    "zkgpu_prof_query": (ctypes.c_int, [ctypes.c_char_p, pu64, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_double)]),
    "zkgpu_prof_kernels": (ctypes.c_int, [ctypes.c_char_p, u64]),
    "zkgpu_mark": (ctypes.c_int, [u32]),
    "zkgpu_mark_elapsed": (ctypes.c_int, [u32, u32, ctypes.POINTER(ctypes.c_double)]),
    # include/zkgpu_parser.h (bindings in zkgpu/parser.py)
    "zkgpu_parser_convert": (ctypes.c_int, [u32, vp, u64, vp, u64, vp, u32, u32, u32, vp]),
    "zkgpu_steps_parser_eval": (ctypes.c_int, [u32, vp, u64, vp, u64, vp, u32, u32, u32, vp]),
    "zkgpu_steps_mirror": (ctypes.c_int, [ctypes.c_int]),
    "zkgpu_steps_invalidate": (ctypes.c_int, [vp]),
    "zkgpu_steps_release_mirrors": (None, []),
    "zkgpu_steps_mirror_bytes": (u64, []),
}


def build():
    """Compile libzkgpu for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", "-C", PKG_ROOT, "-j8"])
    return LIB_PATH


def _absent(name):
    def call(*_):
        raise ZkgpuError("%s is not exported by %s (an older build)" % (name, LIB_PATH))
    return call


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ZkgpuError("libzkgpu.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
        # One HIP runtime per process: torch ships its own libamdhip64.so.7
        # (same SONAME as /opt/rocm's).  Loading torch first makes the dynamic
        # linker bind libzkgpu to that copy, so device pointers and streams
        # are shared; loading ours first would bring up a second runtime.
        try:
            import torch  # noqa: F401
            if torch.version.hip is not None:
                torch.cuda.device_count()
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name, None)
            if f is None:  # an older build (A/B runs, ZKGPU_LIB_DIR): the entry point fails when called
                setattr(L, name, _absent(name))
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def _check(rc, what):
    if rc != 0:
        msg = lib().zkgpu_last_error().decode(errors="replace")
        raise ZkgpuError("%s failed (%d): %s" % (what, rc, msg))


def init(device=0):
    _check(lib().zkgpu_init(device), "zkgpu_init")


def release():
    lib().zkgpu_release()


def set_stream(stream):
    """stream: a torch.cuda.Stream, an int handle, or None (null stream)."""
    h = 0
    if stream is not None:
        h = getattr(stream, "cuda_stream", stream)
    _check(lib().zkgpu_set_stream(h or None), "zkgpu_set_stream")


def synchronize():
    _check(lib().zkgpu_synchronize(), "zkgpu_synchronize")


def _np(a):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return a


def _addr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(type(x))


# ---------------------------------------------------------------- host-pointer
def ntt(x, inverse=False):
    x = _np(x)
    n = x.shape[0]
    ncols = 1 if x.ndim == 1 else x.shape[1]
    out = np.empty_like(x)
    _check(lib().zkgpu_gl_ntt(out.ctypes.data, x.ctypes.data, n, ncols, int(inverse)), "zkgpu_gl_ntt")
    return out


def extend_pol(x, n_ext):
    x = _np(x)
    n = x.shape[0]
    ncols = 1 if x.ndim == 1 else x.shape[1]
    out = np.empty((n_ext,) if x.ndim == 1 else (n_ext, ncols), np.uint64)
    _check(lib().zkgpu_gl_extend_pol(out.ctypes.data, x.ctypes.data, n_ext, n, ncols), "zkgpu_gl_extend_pol")
    return out


def poseidon_full(x):
    x = _np(x)
    out = np.zeros(12, np.uint64)
    _check(lib().zkgpu_gl_poseidon_full(out.ctypes.data, x.ctypes.data), "zkgpu_gl_poseidon_full")
    return out


def poseidon_full_host(x):
    """PoseidonGoldilocks::hash_full_result on the host (the transcript's)."""
    x = _np(x)
    out = np.zeros(12, np.uint64)
    _check(lib().zkgpu_gl_poseidon_full_host(out.ctypes.data, x.ctypes.data), "zkgpu_gl_poseidon_full_host")
    return out


def poseidon_hash(x):
    x = _np(x)
    out = np.zeros(4, np.uint64)
    _check(lib().zkgpu_gl_poseidon_hash(out.ctypes.data, x.ctypes.data), "zkgpu_gl_poseidon_hash")
    return out


def linear_hash(x):
    x = _np(x).reshape(-1)
    out = np.zeros(4, np.uint64)
    buf = x if x.size else np.zeros(1, np.uint64)
    _check(lib().zkgpu_gl_linear_hash(out.ctypes.data, buf.ctypes.data, x.size), "zkgpu_gl_linear_hash")
    return out


def merkle_num_elements(nrows):
    return lib().zkgpu_gl_merkle_num_elements(nrows)


def merkletree(src):
    src = _np(src)
    nrows = src.shape[0]
    ncols = src.shape[1] if src.ndim == 2 else 1
    nodes = np.zeros(merkle_num_elements(nrows), np.uint64)
    buf = src if src.size else np.zeros(1, np.uint64)
    _check(lib().zkgpu_gl_merkletree(nodes.ctypes.data, buf.ctypes.data, ncols, nrows), "zkgpu_gl_merkletree")
    return nodes


def build_const_tree(const_pols, n_bits_ext):
    """bctree: [nPols, nExt, LDE row-major, Merkle nodes] (build_const_tree.cpp:553-603)."""
    x = _np(const_pols)
    n = x.shape[0]
    n_pols = x.shape[1] if x.ndim == 2 else 1
    n_bits = n.bit_length() - 1
    assert 1 << n_bits == n, "rows must be a power of two"
    out = np.zeros(lib().zkgpu_const_tree_num_elements(n_pols, n_bits_ext), np.uint64)
    buf = x if x.size else np.zeros(1, np.uint64)
    _check(lib().zkgpu_build_const_tree(out.ctypes.data, buf.ctypes.data, n_pols, n_bits, n_bits_ext),
           "zkgpu_build_const_tree")
    return out


# ---------------------------------------------------------------- device
def load_rows_dev(cols, ld, rows, block_rows=0, register_host=False):
    """Executor hand-off: host row-major (nrows x ncols) -> device column-major."""
    rows = np.ascontiguousarray(rows, dtype=np.uint64)
    nrows, ncols = rows.shape
    _check(lib().zkgpu_load_rows_dev(_addr(cols), ld, rows.ctypes.data, nrows, ncols, block_rows,
                                     int(register_host)), "zkgpu_load_rows_dev")


class RowsLoad:
    """Background hand-off (zkgpu_load_rows_async): wait() returns once the
    columns hold the rows.  Keeps the host rows and the staging buffer alive
    until then; dropping the object without wait() waits in the finalizer
    (the loader thread still reads `rows` and writes `cols` / `stage`)."""

    def __init__(self, cols, ld, rows, stage, ticket):
        self.cols, self.rows, self.stage, self.ticket = cols, rows, stage, ticket

    def wait(self):
        if self.ticket is not None:
            t, self.ticket = self.ticket, None
            _check(lib().zkgpu_load_wait(t), "zkgpu_load_wait")

    def __del__(self):
        t, self.ticket = getattr(self, "ticket", None), None
        if t is not None and _lib is not None:
            _lib.zkgpu_load_wait(t)  # status dropped: nobody is left to receive it


def load_rows_async(cols, ld, rows, stage, block_rows=0):
    """Start the load of host row-major rows into device column-major cols on
    the library's loader thread; stage: device buffer of at least
    load_rows_stage_bytes(nrows, ncols) bytes.  Returns a RowsLoad."""
    rows = np.ascontiguousarray(rows, dtype=np.uint64)
    nrows, ncols = rows.shape
    t = ctypes.c_void_p()
    _check(lib().zkgpu_load_rows_async(_addr(cols), ld, rows.ctypes.data, nrows, ncols, block_rows, _addr(stage),
                                       stage.numel() * stage.element_size(), ctypes.byref(t)), "zkgpu_load_rows_async")
    return RowsLoad(cols, ld, rows, stage, t)


def load_rows_stage_bytes(nrows, ncols, block_rows=0):
    return int(lib().zkgpu_load_rows_stage_bytes(nrows, ncols, block_rows))


def ntt_dev(dst, ld_dst, src, ld_src, n, ncols, inverse=False):
    _check(lib().zkgpu_gl_ntt_dev(_addr(dst), ld_dst, _addr(src), ld_src, n, ncols, int(inverse)), "zkgpu_gl_ntt_dev")


def extend_pol_dev(out, ld_out, src, ld_in, n_ext, n, ncols):
    _check(lib().zkgpu_gl_extend_pol_dev(_addr(out), ld_out, _addr(src), ld_in, n_ext, n, ncols),
           "zkgpu_gl_extend_pol_dev")


def extend_pol_inplace_dev(base, n_ext, n, ncols):
    """extendPol in place: base holds ncols n-row columns (ld n) on entry and
    their n_ext-row extensions (ld n_ext) on return"""
    _check(lib().zkgpu_gl_extend_pol_inplace_dev(_addr(base), n_ext, n, ncols), "zkgpu_gl_extend_pol_inplace_dev")


def set_lde_batch_cols(max_cols):
    """at most max_cols columns per extend_pol batch (0: the default)"""
    lib().zkgpu_set_lde_batch_cols(max_cols)


def rows_to_cols_dev(cols, ld, rows, nrows, ncols):
    _check(lib().zkgpu_rows_to_cols_dev(_addr(cols), ld, _addr(rows), nrows, ncols), "zkgpu_rows_to_cols_dev")


def cols_to_rows_dev(rows, cols, ld, nrows, ncols):
    _check(lib().zkgpu_cols_to_rows_dev(_addr(rows), _addr(cols), ld, nrows, ncols), "zkgpu_cols_to_rows_dev")


def poseidon_batch_dev(out, src, n, full=True):
    _check(lib().zkgpu_gl_poseidon_batch_dev(_addr(out), _addr(src), n, int(full)), "zkgpu_gl_poseidon_batch_dev")


def merkletree_dev(nodes, src, ld, ncols, nrows):
    _check(lib().zkgpu_gl_merkletree_dev(_addr(nodes), _addr(src), ld, ncols, nrows), "zkgpu_gl_merkletree_dev")


def merkletree2_dev(nodes, src, src2, ld, split, ncols, nrows):
    """tree of a section in two regions: columns [0, split) at src, the rest at src2"""
    _check(lib().zkgpu_gl_merkletree2_dev(_addr(nodes), _addr(src), _addr(src2), ld, split, ncols, nrows),
           "zkgpu_gl_merkletree2_dev")


def merkletree_rows_dev(nodes, src, ncols, nrows):
    _check(lib().zkgpu_gl_merkletree_rows_dev(_addr(nodes), _addr(src), ncols, nrows),
           "zkgpu_gl_merkletree_rows_dev")


def merkle_open_dev(nodes, src, ld, ncols, nrows, idx):
    idx = _np(idx).reshape(-1)
    nq = idx.size
    nlev = max(0, int(nrows).bit_length() - 1)
    vals = np.zeros((nq, ncols), np.uint64)
    sibs = np.zeros((nq, nlev, 4), np.uint64)
    _check(lib().zkgpu_gl_merkle_open_dev(vals.ctypes.data, sibs.ctypes.data, _addr(nodes), _addr(src), ld, ncols,
                                          nrows, idx.ctypes.data, nq), "zkgpu_gl_merkle_open_dev")
    return vals, sibs


def fri_fold_dev(out, pol, pol_bits, out_bits, special_x, shift_inv):
    sx = _np(special_x)
    _check(lib().zkgpu_fri_fold_dev(_addr(out), _addr(pol), pol_bits, out_bits, sx.ctypes.data, shift_inv),
           "zkgpu_fri_fold_dev")


def fri_fold_rows_dev(out, rows, g0, ngroups, pol_bits, out_bits, special_x, shift_inv):
    """the fold for output groups [g0, g0 + ngroups) from their getTransposed rows"""
    sx = _np(special_x)
    _check(lib().zkgpu_fri_fold_rows_dev(_addr(out), _addr(rows), g0, ngroups, pol_bits, out_bits, sx.ctypes.data,
                                         shift_inv), "zkgpu_fri_fold_rows_dev")


def fri_transpose_dev(aux, pol, degree, transpose_bits):
    _check(lib().zkgpu_fri_transpose_dev(_addr(aux), _addr(pol), degree, transpose_bits), "zkgpu_fri_transpose_dev")


def field_selftest_dev(out, a, b, n, op):
    _check(lib().zkgpu_gl_field_selftest_dev(_addr(out), _addr(a), _addr(b), n, op), "zkgpu_gl_field_selftest_dev")


def field_selftest_rb_dev(out, a, b, c, n, op, e=0):
    """include/zkgpu.h zkgpu_gl_field_selftest_rb_dev (c may be None)."""
    _check(lib().zkgpu_gl_field_selftest_rb_dev(_addr(out), _addr(a), _addr(b), _addr(c) if c is not None else None,
                                                n, op, e), "zkgpu_gl_field_selftest_rb_dev")


def calculate_z_dev(z, z_ld, num, num_ld, den, den_ld, n):
    closes = ctypes.c_int(0)
    _check(lib().zkgpu_calculate_z_dev(_addr(z), z_ld, _addr(num), num_ld, _addr(den), den_ld, n,
                                       ctypes.byref(closes)), "zkgpu_calculate_z_dev")
    return bool(closes.value)



class ZReq(ctypes.Structure):
    """zkgpu_z_req (include/zkgpu.h)"""
    _fields_ = [("z", vp), ("z_ld", u64), ("num", vp), ("num_ld", u64), ("den", vp), ("den_ld", u64)]


def calculate_z_many_dev(reqs, n):
    """Several grand products in one round trip (zkgpu_calculate_z_many_dev):
    reqs = [(z, z_ld, num, num_ld, den, den_ld)]; returns [closes] per request."""
    arr = (ZReq * max(1, len(reqs)))()
    for k, (z, z_ld, num, num_ld, den, den_ld) in enumerate(reqs):
        arr[k] = ZReq(_addr(z), z_ld, _addr(num), num_ld, _addr(den), den_ld)
    closes = (ctypes.c_int * max(1, len(reqs)))()
    _check(lib().zkgpu_calculate_z_many_dev(arr, len(reqs), n, closes), "zkgpu_calculate_z_many_dev")
    return [bool(closes[k]) for k in range(len(reqs))]


def calculate_z_block_dev(z, z_ld, num, num_ld, den, den_ld, n, z0=(1, 0, 0)):
    """One row block of calculateZ: z = z0 * running product; returns the
    block's closing total z0 * prod(num / den) (3 canonical u64)."""
    z0a = np.array([int(v) for v in z0], dtype=np.uint64)
    tot = np.zeros(3, np.uint64)
    _check(lib().zkgpu_calculate_z_block_dev(_addr(z), z_ld, _addr(num), num_ld, _addr(den), den_ld, n,
                                             z0a.ctypes.data, tot.ctypes.data), "zkgpu_calculate_z_block_dev")
    return tot

def xdivxsub_dev(xdiv, xdivw, xi, n_bits, n_bits_ext):
    x = _np(xi)
    _check(lib().zkgpu_xdivxsub_dev(_addr(xdiv), _addr(xdivw), x.ctypes.data, n_bits, n_bits_ext),
           "zkgpu_xdivxsub_dev")


def xdivxsub_rows_dev(xdiv, xdivw, xi, n_bits, n_bits_ext, row0, nrows):
    """rows [row0, row0 + nrows) of xdivxsub_dev, written at their places"""
    x = _np(xi)
    _check(lib().zkgpu_xdivxsub_rows_dev(_addr(xdiv), _addr(xdivw), x.ctypes.data, n_bits, n_bits_ext, row0, nrows),
           "zkgpu_xdivxsub_rows_dev")


def lagrange_xi_rows_dev(lev, lpev, ld, xi, n_bits, row0, nrows):
    """LEv / LpEv rows [row0, row0 + nrows) in closed form (3 columns of
    leading dimension ld each, row row0 at offset 0)"""
    x = _np(xi)
    _check(lib().zkgpu_lagrange_xi_rows_dev(_addr(lev), _addr(lpev), ld, x.ctypes.data, n_bits, row0, nrows),
           "zkgpu_lagrange_xi_rows_dev")


def ext_powers_dev(out, ld, base, n):
    b = _np(base)
    _check(lib().zkgpu_ext_powers_dev(_addr(out), ld, b.ctypes.data, n), "zkgpu_ext_powers_dev")


class Sections(ctypes.Structure):
    """zkgpu_sections (include/zkgpu.h): 12 column-major section bases."""
    _fields_ = [("sec", vp * 12), ("ld", u64 * 12), ("ncols", u32 * 12)]


def zxp_eval_dev(prog, sections, log_dom, challenges, publics, evals=None, xdiv=None, xdivw=None, extend_bits=0,
                 x_start=1):
    """Evaluate one ZXP program (zkgpu.synthetic.Program or (instr, opnd,
    n_tmp1, n_tmp3)) over the domain; sections: {index: (tensor, ld, ncols)}."""
    if hasattr(prog, "arrays"):
        ins, opn = prog.arrays()
        nt1, nt3 = prog.n_tmp1, prog.n_tmp3
    else:
        ins, opn, nt1, nt3 = prog
    ins = np.ascontiguousarray(ins, np.uint32)
    opn = np.ascontiguousarray(opn, np.uint32)
    s = Sections()
    for k, (t, ld, nc) in sections.items():
        s.sec[k] = _addr(t)
        s.ld[k] = ld
        s.ncols[k] = nc
    ch = np.zeros(24, np.uint64)
    c = _np(challenges).reshape(-1)
    ch[:c.size] = c
    pub = _np(publics if publics is not None else np.zeros(1, np.uint64))
    ev = _np(evals if evals is not None else np.zeros(3, np.uint64)).reshape(-1)
    _check(lib().zkgpu_zxp_eval_dev(ins.ctypes.data, ins.shape[0], opn.ctypes.data, opn.shape[0], max(nt1, 1),
                                    max(nt3, 1), ctypes.byref(s), log_dom, ch.ctypes.data, pub.ctypes.data,
                                    pub.size if publics is not None else 0, ev.ctypes.data, ev.size // 3,
                                    _addr(xdiv), _addr(xdivw), extend_bits, x_start), "zkgpu_zxp_eval_dev")


class ZxpCompiled(ctypes.Structure):
    """zxp_compiled (include/zkgpu_zxp.h)."""
    _fields_ = [("instr", vp), ("n_instr", u32), ("opnd", vp), ("n_opnd", u32), ("term", vp), ("n_term", u32),
                ("cst", vp), ("n_cst", u32), ("n_tmp1", u32), ("n_tmp3", u32)]


ZXP_TERM_DTYPE = np.dtype([("src", np.uint32), ("comp", np.uint32), ("coef", np.uint64, 3)])


def zxp_compile(prog, challenges, publics, evals=None, max_terms=0):
    """Host-only compile of a ZXP program (zkgpu_zxp_compile, no GPU needed).
    Returns dict(instr, opnd, term, cst, n_tmp1, n_tmp3) of numpy copies."""
    ins, opn = prog.arrays()
    ins = np.ascontiguousarray(ins, np.uint32)
    opn = np.ascontiguousarray(opn, np.uint32)
    ch = np.zeros(24, np.uint64)
    c = _np(challenges).reshape(-1)
    ch[:c.size] = c
    pub = _np(publics if publics is not None else np.zeros(1, np.uint64))
    ev = _np(evals if evals is not None else np.zeros(3, np.uint64)).reshape(-1)
    out = ZxpCompiled()
    _check(lib().zkgpu_zxp_compile(ins.ctypes.data, ins.shape[0], opn.ctypes.data, opn.shape[0],
                                   max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ch.ctypes.data, pub.ctypes.data,
                                   pub.size if publics is not None else 0, ev.ctypes.data, ev.size // 3, max_terms,
                                   ctypes.byref(out)), "zkgpu_zxp_compile")

    def grab(ptr, n, dtype, width):
        if n == 0:
            return np.zeros((0, width) if width else 0, dtype)
        nbytes = n * (width or 1) * np.dtype(dtype).itemsize
        a = np.frombuffer(ctypes.string_at(ptr, nbytes), dtype=dtype).copy()
        return a.reshape(n, width) if width else a

    return {"instr": grab(out.instr, out.n_instr, np.uint32, 4), "opnd": grab(out.opnd, out.n_opnd, np.uint32, 4),
            "term": grab(out.term, out.n_term, ZXP_TERM_DTYPE, 0), "cst": grab(out.cst, out.n_cst, np.uint64, 3),
            "n_tmp1": out.n_tmp1, "n_tmp3": out.n_tmp3}


def zxp_jit_source(prog, challenges, publics, evals=None, rtc_check=False):
    """Generated straight-line kernel source of a program (zkgpu_zxp_jit_source,
    no GPU needed); with rtc_check, also compiled for gfx950 by hiprtc."""
    ins, opn = prog.arrays()
    ins = np.ascontiguousarray(ins, np.uint32)
    opn = np.ascontiguousarray(opn, np.uint32)
    ch = np.zeros(24, np.uint64)
    c = _np(challenges).reshape(-1)
    ch[:c.size] = c
    pub = _np(publics if publics is not None else np.zeros(1, np.uint64))
    ev = _np(evals if evals is not None else np.zeros(3, np.uint64)).reshape(-1)
    size = 1 << 22
    while True:  # the return value is the source length: grow the buffer until it fits
        buf = ctypes.create_string_buffer(size)
        rc = lib().zkgpu_zxp_jit_source(ins.ctypes.data, ins.shape[0], opn.ctypes.data, opn.shape[0],
                                        max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ch.ctypes.data, pub.ctypes.data,
                                        pub.size if publics is not None else 0, ev.ctypes.data, ev.size // 3,
                                        buf, len(buf), int(rtc_check))
        if rc < 0:
            _check(rc, "zkgpu_zxp_jit_source")
        if rc < size:
            return buf.value.decode()
        size = rc + 1
        rtc_check = False  # compiled (or cached) already


def zxp_jit_cached(prog, challenges, publics, evals=None):
    """True when the program's compiled kernel is in the on-disk cache
    (zkgpu_zxp_jit_source with rtc_check = 3; no compile, no GPU)."""
    ins, opn = prog.arrays()
    ins = np.ascontiguousarray(ins, np.uint32)
    opn = np.ascontiguousarray(opn, np.uint32)
    ch = np.zeros(24, np.uint64)
    c = _np(challenges).reshape(-1)
    ch[:c.size] = c
    pub = _np(publics if publics is not None else np.zeros(1, np.uint64))
    ev = _np(evals if evals is not None else np.zeros(3, np.uint64)).reshape(-1)
    rc = lib().zkgpu_zxp_jit_source(ins.ctypes.data, ins.shape[0], opn.ctypes.data, opn.shape[0],
                                    max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ch.ctypes.data, pub.ctypes.data,
                                    pub.size if publics is not None else 0, ev.ctypes.data, ev.size // 3,
                                    None, 0, 3)
    if rc < 0:
        _check(rc, "zkgpu_zxp_jit_source")
    return rc == 1


def zxp_eval_block_dev(prog, sections, log_rows, log_domain, challenges, publics, evals=None, xdiv=None, xdivw=None,
                       extend_bits=0, x_start=7):
    """One row block of a row-sharded domain (zkgpu_zxp_eval_block_dev):
    sections carry the block plus halo rows; x_start = 7 * w^row0."""
    ins, opn = prog.arrays()
    ins = np.ascontiguousarray(ins, np.uint32)
    opn = np.ascontiguousarray(opn, np.uint32)
    s = Sections()
    for k, (t, ld, nc) in sections.items():
        s.sec[k] = _addr(t)
        s.ld[k] = ld
        s.ncols[k] = nc
    ch = np.zeros(24, np.uint64)
    c = _np(challenges).reshape(-1)
    ch[:c.size] = c
    pub = _np(publics if publics is not None else np.zeros(1, np.uint64))
    ev = _np(evals if evals is not None else np.zeros(3, np.uint64)).reshape(-1)
    _check(lib().zkgpu_zxp_eval_block_dev(ins.ctypes.data, ins.shape[0], opn.ctypes.data, opn.shape[0],
                                          max(prog.n_tmp1, 1), max(prog.n_tmp3, 1), ctypes.byref(s), log_rows,
                                          log_domain, ch.ctypes.data, pub.ctypes.data,
                                          pub.size if publics is not None else 0, ev.ctypes.data, ev.size // 3,
                                          _addr(xdiv), _addr(xdivw), extend_bits, x_start),
           "zkgpu_zxp_eval_block_dev")


def merkle_open_rows_dev(nodes, src, ncols, nrows, idx):
    """MerkleTreeGL::getGroupProof for a row-major device source."""
    idx = _np(idx).reshape(-1)
    nq = idx.size
    nlev = max(0, int(nrows).bit_length() - 1)
    vals = np.zeros((nq, ncols), np.uint64)
    sibs = np.zeros((nq, nlev, 4), np.uint64)
    _check(lib().zkgpu_gl_merkle_open_rows_dev(vals.ctypes.data, sibs.ctypes.data, _addr(nodes), _addr(src), ncols,
                                               nrows, idx.ctypes.data, nq), "zkgpu_gl_merkle_open_rows_dev")
    return vals, sibs


class OpenReq(ctypes.Structure):
    """zkgpu_open_req (include/zkgpu.h)"""
    _fields_ = [("vals_out", vp), ("sibs_out", vp), ("nodes", vp), ("src", vp), ("ld", u64), ("ncols", u64),
                ("nrows", u64), ("idx", vp), ("nq", u64), ("rows", u32)]


def merkle_open_many(reqs):
    """Several trees' openings in one round trip (zkgpu_gl_merkle_open_many).
    reqs: (nodes, src, ld, ncols, nrows, idx, rows) per tree -- rows=False is
    merkle_open_dev's column-major source (ld), rows=True merkle_open_rows_dev's
    row-major one.  Returns [(vals, sibs)] in request order."""
    out, keep = [], []
    arr = (OpenReq * max(1, len(reqs)))()
    for k, (nodes, src, ld, ncols, nrows, idx, rows) in enumerate(reqs):
        idx = np.ascontiguousarray(_np(idx).reshape(-1))
        nlev = max(0, int(nrows).bit_length() - 1)
        vals = np.zeros((idx.size, ncols), np.uint64)
        sibs = np.zeros((idx.size, nlev, 4), np.uint64)
        keep.append(idx)
        out.append((vals, sibs))
        arr[k] = OpenReq(vals.ctypes.data, sibs.ctypes.data, _addr(nodes), _addr(src), ld, ncols, nrows,
                         idx.ctypes.data, idx.size, 1 if rows else 0)
    _check(lib().zkgpu_gl_merkle_open_many(arr, len(reqs)), "zkgpu_gl_merkle_open_many")
    return out


def h1h2_dev(h1, h1_ld, h2, h2_ld, f, f_ld, t, t_ld, n, dim):
    """Plookup h1/h2 on device columns.  Returns None, or the first f row whose
    value is not in t (the call then fails with "Number not included")."""
    miss = ctypes.c_uint64(0)
    rc = lib().zkgpu_h1h2_dev(_addr(h1), h1_ld, _addr(h2), h2_ld, _addr(f), f_ld, _addr(t), t_ld, n, dim,
                              ctypes.byref(miss))
    if rc != 0 and miss.value != (1 << 64) - 1:
        return miss.value
    _check(rc, "zkgpu_h1h2_dev")
    return None


# calculateH1H2 over row-sharded f / t (include/zkgpu.h zkgpu_h1h2_shard_*;
# host/sharded_starks.hpp h1h2_sharded runs the same steps with exchanges)
def h1h2_shard_route(recs, cap, f, f_ld, t, t_ld, nrows, row0, dim, world):
    """-> (n_t, n_f): the rank's bucket sizes per owner"""
    nt = np.zeros(world, np.uint32)
    nf = np.zeros(world, np.uint32)
    _check(lib().zkgpu_h1h2_shard_route(_addr(recs), cap, nt.ctypes.data, nf.ctypes.data, _addr(f), f_ld, _addr(t),
                                        t_ld, nrows, row0, dim, world), "zkgpu_h1h2_shard_route")
    return nt, nf


def h1h2_shard_owner(ret, recs, nrec, dim):
    """-> the smallest f row without a table row, or None"""
    miss = ctypes.c_uint64(0)
    _check(lib().zkgpu_h1h2_shard_owner(_addr(ret), _addr(recs), nrec, dim, ctypes.byref(miss)),
           "zkgpu_h1h2_shard_owner")
    return None if miss.value == (1 << 64) - 1 else miss.value


def h1h2_shard_counts(start, cnt, sent, ret, nsent, nrows, row0):
    """-> the rank's multiset total"""
    tot = ctypes.c_uint64(0)
    _check(lib().zkgpu_h1h2_shard_counts(_addr(start), _addr(cnt), ctypes.byref(tot), _addr(sent), _addr(ret), nsent,
                                         nrows, row0), "zkgpu_h1h2_shard_counts")
    return tot.value


def h1h2_shard_deal(seg, seg_ld, t, t_ld, start, cnt, nrows, dim):
    _check(lib().zkgpu_h1h2_shard_deal(_addr(seg), seg_ld, _addr(t), t_ld, _addr(start), _addr(cnt), nrows, dim),
           "zkgpu_h1h2_shard_deal")


def h1h2_shard_place(h1, h1_ld, h2, h2_ld, buf, buf_ld, pos0, length, row0, dim):
    _check(lib().zkgpu_h1h2_shard_place(_addr(h1), h1_ld, _addr(h2), h2_ld, _addr(buf), buf_ld, pos0, length, row0,
                                        dim), "zkgpu_h1h2_shard_place")


def qsplit_dev(qq2, ld2, qq1, ld1, n, q_deg, shift_in):
    _check(lib().zkgpu_qsplit_dev(_addr(qq2), ld2, _addr(qq1), ld1, n, q_deg, shift_in), "zkgpu_qsplit_dev")


def qsplit_cols_dev(qq2, ld2, qq1, ld1, n, q_deg, shift_in, dim, stride):
    _check(lib().zkgpu_qsplit_cols_dev(_addr(qq2), ld2, _addr(qq1), ld1, n, q_deg, shift_in, dim, stride),
           "zkgpu_qsplit_cols_dev")


def evmap_dev(cols, lds, dims, primes, lev, lpev, l_ld, n, extend_bits):
    n_ev = len(cols)
    ptrs = (ctypes.c_void_p * n_ev)(*[_addr(c) for c in cols])
    lds_a = _np(lds)
    dims_a = np.ascontiguousarray(dims, np.uint32)
    pr_a = np.ascontiguousarray(primes, np.uint32)
    out = np.zeros((n_ev, 3), np.uint64)
    _check(lib().zkgpu_evmap_dev(out.ctypes.data, ctypes.cast(ptrs, ctypes.c_void_p), lds_a.ctypes.data,
                                 dims_a.ctypes.data, pr_a.ctypes.data, n_ev, _addr(lev), _addr(lpev), l_ld, n,
                                 extend_bits), "zkgpu_evmap_dev")
    return out


# ---------------------------------------------------------------- profiling
def prof_enable(on=True):
    _check(lib().zkgpu_prof_enable(int(on)), "zkgpu_prof_enable")


def prof_reset():
    _check(lib().zkgpu_prof_reset(), "zkgpu_prof_reset")


def prof_query(kernel):
    """-> (launches, total_ms, total_algorithmic_bytes) since the last reset."""
    n = ctypes.c_uint64(0)
    ms = ctypes.c_double(0)
    by = ctypes.c_double(0)
    _check(lib().zkgpu_prof_query(kernel.encode(), ctypes.byref(n), ctypes.byref(ms), ctypes.byref(by)),
           "zkgpu_prof_query")
    return n.value, ms.value, by.value


def prof_kernels():
    buf = ctypes.create_string_buffer(4096)
    _check(lib().zkgpu_prof_kernels(buf, len(buf)), "zkgpu_prof_kernels")
    return [k for k in buf.value.decode().split("\n") if k]


# ---------------------------------------------------------------- torch helpers
def to_device(a, device="cuda:0"):
    """numpy uint64 -> torch int64 tensor on the GPU (bit-identical storage)."""
    import torch
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return torch.from_numpy(a.view(np.int64)).to(device)


def from_device(t):
    return t.detach().cpu().numpy().view(np.uint64)
