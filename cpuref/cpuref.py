"""cpuref/cpuref.py -- bench.py's CPU baseline only (not the checker, not the
product): ctypes wrapper of libcpuref.so, the reference's AVX2 + OpenMP CPU
path for the proof's bulk kernels restated (cpuref.cpp), with the oracle's
row-major conventions (oracle/oracle.py)."""
import contextlib
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "libcpuref.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(path)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.cr_merkletree.argtypes = [vp, vp, u64, u64]
        L.cr_merkletree.restype = None
        L.cr_extend_pol.argtypes = [vp, vp, u64, u64, u64]
        L.cr_extend_pol.restype = None
        L.cr_ntt.argtypes = [vp, vp, u64, u64, ctypes.c_int]
        L.cr_ntt.restype = None
        L.cr_merkle_num_elements.argtypes = [u64]
        L.cr_merkle_num_elements.restype = u64
        L.cr_set_num_threads.argtypes = [ctypes.c_int]
        L.cr_set_num_threads.restype = None
        L.cr_num_threads.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _u64(x):
    return np.ascontiguousarray(x, dtype=np.uint64)


def extend_pol(x, n_ext):
    x = _u64(x)
    n = x.shape[0]
    ncols = 1 if x.ndim == 1 else x.shape[1]
    out = np.empty((n_ext,) if x.ndim == 1 else (n_ext, ncols), np.uint64)
    lib().cr_extend_pol(out.ctypes.data, x.ctypes.data, n_ext, n, ncols)
    return out


def ntt(x, inverse=False):
    x = _u64(x)
    out = np.empty_like(x)
    lib().cr_ntt(out.ctypes.data, x.ctypes.data, x.shape[0], 1 if x.ndim == 1 else x.shape[1], int(inverse))
    return out


def merkletree(src):
    src = _u64(src)
    nrows = src.shape[0]
    ncols = src.shape[1] if src.ndim == 2 else 1
    out = np.zeros(lib().cr_merkle_num_elements(nrows), np.uint64)
    lib().cr_merkletree(out.ctypes.data, src.ctypes.data, ncols, nrows)
    return out


class _OracleLibWithSteps:
    """the oracle's ctypes library with oc_zxp_eval (the Steps programs)
    answered by cr_zxp_eval (same contract, 4 rows per AVX2 step)"""

    def __init__(self, olib):
        self._o = olib
        f = lib().cr_zxp_eval
        f.argtypes = olib.oc_zxp_eval.argtypes
        f.restype = None
        self.oc_zxp_eval = f

    def __getattr__(self, name):
        return getattr(self._o, name)


@contextlib.contextmanager
def as_oracle_kernels(oc):
    """the oracle prover (oracle/stark_prover.py) with its LDE, NTT, Merkle
    and Steps-program kernels taken from cpuref -- the proof is unchanged
    (bit-identical kernels, tests/test_cpuref.py); used to time the
    reference's CPU path (bench.py cpu_baseline)"""
    saved = oc.extend_pol, oc.ntt, oc.merkletree, oc.lib
    proxy = _OracleLibWithSteps(oc.lib())
    oc.extend_pol, oc.ntt, oc.merkletree, oc.lib = extend_pol, ntt, merkletree, (lambda: proxy)
    try:
        yield
    finally:
        oc.extend_pol, oc.ntt, oc.merkletree, oc.lib = saved
