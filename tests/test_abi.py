"""CPU-side checks of the product library: it builds for gfx950, loads, and
exports every entry point include/zkgpu.h declares (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols(name="zkgpu.h"):
    text = open(os.path.join(ROOT, "include", name)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(zkgpu_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    import zkgpu
    if not os.path.exists(zkgpu.LIB_PATH):
        zkgpu.build()
    L = ctypes.CDLL(zkgpu.LIB_PATH)
    syms = sorted(header_symbols("zkgpu.h") + header_symbols("zkgpu_parser.h"))
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # the Python binding covers the whole ABI
    assert sorted(zkgpu.exported_symbols()) == syms


def test_stark_library_exports_every_declared_symbol():
    """include/zkgpu_stark.h is libzkgpu_stark.so (host/starks.cpp)."""
    import zkgpu
    from zkgpu import stark
    L = ctypes.CDLL(stark.STARK_LIB)
    syms = header_symbols("zkgpu_stark.h")
    assert len(syms) >= 8
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_every_header_is_checked():
    names = sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h"))
    assert set(names) <= {"zkgpu.h", "zkgpu_parser.h", "zkgpu_stark.h", "zkgpu_zxp.h"}, names


def test_library_has_gfx950_code_object():
    import zkgpu
    data = open(zkgpu.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_calls_fail_loudly_without_init():
    """No silent CPU path: a compute call before zkgpu_init is an error."""
    import zkgpu
    import numpy as np
    with pytest.raises(zkgpu.ZkgpuError):
        zkgpu.ntt(np.arange(16, dtype=np.uint64))


def test_host_permutation_vs_oracle(oracle):
    """The transcript's host permutation (zkgpu_gl_poseidon_full_host: full
    rounds + the sparse partial rounds of poseidon_gl_sparse.h) equals the
    oracle's textbook permutation, non-canonical inputs included.  CPU only."""
    import numpy as np
    import zkgpu
    P = 0xFFFFFFFF00000001
    rng = np.random.default_rng(77)
    cases = [np.zeros(12, np.uint64), np.full(12, P - 1, np.uint64), np.full(12, 2**64 - 1, np.uint64),
             np.arange(12, dtype=np.uint64) + np.uint64(P - 6)]
    cases += [rng.integers(0, 2**64 - 1, 12, dtype=np.uint64, endpoint=True) for _ in range(200)]
    for x in cases:
        assert np.array_equal(zkgpu.poseidon_full_host(x), oracle.poseidon_full(x % np.uint64(P))), x
