"""Python binding of include/zkgpu_parser.h: the reference's Steps bytecode
(zkevm.chelpers.<step>.parser.hpp op*/args*) converted to ZXP programs and
evaluated on the GPU.  Used by the tests and bench.py; the host C++ adapter is
host/zkgpu_steps.hpp."""
import ctypes

import numpy as np

from . import ZkgpuError, lib, _check

STEP2PREV, STEP3PREV, STEP3, STEP42NS, STEP52NS = range(5)
NAMES = ["step2prev", "step3prev", "step3", "step42ns", "step52ns"]


class PolsSection(ctypes.Structure):
    _fields_ = [("section", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("offset", ctypes.c_uint64),
                ("width", ctypes.c_uint64)]


class _ZxpProgram(ctypes.Structure):
    _fields_ = [("instr", ctypes.c_void_p), ("n_instr", ctypes.c_uint32), ("opnd", ctypes.c_void_p),
                ("n_opnd", ctypes.c_uint32), ("n_tmp1", ctypes.c_uint32), ("n_tmp3", ctypes.c_uint32),
                ("domain_ext", ctypes.c_uint32)]


class StepsParams(ctypes.Structure):
    _fields_ = [("pols", ctypes.c_void_p), ("const_pols", ctypes.c_void_p), ("n_const", ctypes.c_uint64),
                ("challenges", ctypes.c_void_p), ("evals", ctypes.c_void_p), ("n_evals", ctypes.c_uint32),
                ("n_publics", ctypes.c_uint32), ("publics", ctypes.c_void_p), ("xdiv", ctypes.c_void_p),
                ("xdivw", ctypes.c_void_p), ("q_2ns", ctypes.c_void_p), ("f_2ns", ctypes.c_void_p)]


class Converted:
    """A ZXP program produced from bytecode (the .arrays() / n_tmp* / domain_ext
    interface of zkgpu.synthetic.Program)."""

    def __init__(self, instr, opnd, n_tmp1, n_tmp3, domain_ext):
        self.instr_arr, self.opnd_arr = instr, opnd
        self.n_tmp1, self.n_tmp3, self.domain_ext = n_tmp1, n_tmp3, domain_ext
        self.instr = [tuple(int(x) for x in r) for r in instr]
        self.opnd = [tuple(int(x) for x in r) for r in opnd]

    def arrays(self):
        return self.instr_arr, self.opnd_arr


def sections_array(sections):
    """[(zxp section, offset, width), ...] -> ctypes array"""
    arr = (PolsSection * max(len(sections), 1))()
    for k, (sec, off, w) in enumerate(sections):
        arr[k].section, arr[k].offset, arr[k].width = sec, off, w
    return arr


def convert(parser, ops, args, sections, n_bits, n_bits_ext):
    ops = np.ascontiguousarray(ops, np.uint64)
    args = np.ascontiguousarray(args, np.uint64)
    secs = sections_array(sections)
    out = _ZxpProgram()
    _check(lib().zkgpu_parser_convert(parser, ops.ctypes.data, ops.size, args.ctypes.data, args.size, secs,
                                      len(sections), n_bits, n_bits_ext, ctypes.byref(out)), "zkgpu_parser_convert")
    ins = np.frombuffer(ctypes.string_at(out.instr, out.n_instr * 16), np.uint32).reshape(-1, 4).copy()
    opn = np.frombuffer(ctypes.string_at(out.opnd, out.n_opnd * 16), np.uint32).reshape(-1, 4).copy()
    return Converted(ins, opn, out.n_tmp1, out.n_tmp3, out.domain_ext)


def steps_eval(parser, ops, args, sections, n_bits, n_bits_ext, pols, const_pols, challenges, publics=None,
               evals=None, xdiv=None, xdivw=None, q_2ns=None, f_2ns=None):
    """zkgpu_steps_parser_eval on host numpy buffers (pols: the flat memory map
    as a 1-D uint64 array whose sections start at their offsets; outputs are
    written in place)."""
    ops = np.ascontiguousarray(ops, np.uint64)
    args = np.ascontiguousarray(args, np.uint64)
    secs = sections_array(sections)
    keep = []

    def ptr(a):
        if a is None:
            return None
        assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
        keep.append(a)
        return a.ctypes.data

    p = StepsParams()
    p.pols = ptr(pols)
    p.const_pols = ptr(const_pols)
    p.n_const = const_pols.shape[1] if const_pols is not None else 0
    p.challenges = ptr(np.ascontiguousarray(challenges, np.uint64).reshape(-1))
    if evals is not None:
        ev = np.ascontiguousarray(evals, np.uint64).reshape(-1)
        p.evals, p.n_evals = ptr(ev), ev.size // 3
    if publics is not None:
        pu = np.ascontiguousarray(publics, np.uint64)
        p.publics, p.n_publics = ptr(pu), pu.size
    p.xdiv, p.xdivw, p.q_2ns, p.f_2ns = ptr(xdiv), ptr(xdivw), ptr(q_2ns), ptr(f_2ns)
    rc = lib().zkgpu_steps_parser_eval(parser, ops.ctypes.data, ops.size, args.ctypes.data, args.size, secs,
                                       len(sections), n_bits, n_bits_ext, ctypes.byref(p))
    if rc:
        raise ZkgpuError("zkgpu_steps_parser_eval failed (%d): %s"
                         % (rc, lib().zkgpu_last_error().decode(errors="replace")))
