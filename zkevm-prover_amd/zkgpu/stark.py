"""Python binding of libzkgpu_stark (host/starks.cpp): the GPU STARK prover.

Builds the zkgpu_stark_info description (include/zkgpu_stark.h) from a
SyntheticStark instance, runs setup / witness / prove, and returns the proof
in the reference's zkin layout with canonical decimal strings (the same form
as the reference's testvectors and the oracle's prover).
"""
import ctypes
import os

import numpy as np

from . import ZkgpuError, lib as _zk_lib

_HERE = os.path.dirname(os.path.abspath(__file__))
STARK_LIB = os.path.join(os.environ.get("ZKGPU_LIB_DIR") or os.path.join(os.path.dirname(_HERE), "lib"),
                         "libzkgpu_stark.so")
P = 0xFFFFFFFF00000001


class _Prog(ctypes.Structure):
    _fields_ = [("instr", ctypes.c_void_p), ("n_instr", ctypes.c_uint32), ("opnd", ctypes.c_void_p),
                ("n_opnd", ctypes.c_uint32), ("n_tmp1", ctypes.c_uint32), ("n_tmp3", ctypes.c_uint32)]


class _Info(ctypes.Structure):
    _fields_ = [("n_bits", ctypes.c_uint32), ("n_bits_ext", ctypes.c_uint32), ("n_queries", ctypes.c_uint32),
                ("n_fri_steps", ctypes.c_uint32), ("fri_steps", ctypes.c_uint32 * 32),
                ("n_cm1", ctypes.c_uint32), ("n_cm2", ctypes.c_uint32), ("n_cm3", ctypes.c_uint32),
                ("n_cm4", ctypes.c_uint32), ("n_tmp", ctypes.c_uint32), ("n_const", ctypes.c_uint32),
                ("n_publics", ctypes.c_uint32), ("q_deg", ctypes.c_uint32), ("l_first", ctypes.c_uint32),
                ("n_k", ctypes.c_uint32), ("seed", ctypes.c_uint64),
                ("n_random_cols", ctypes.c_uint32), ("random_cols", ctypes.c_void_p),
                ("n_zctx", ctypes.c_uint32), ("zctx", ctypes.c_void_p),
                ("n_ev", ctypes.c_uint32), ("ev", ctypes.c_void_p),
                ("step1", _Prog), ("step2", _Prog), ("step3prev", _Prog), ("step42ns", _Prog), ("step52ns", _Prog),
                ("n_random_const", ctypes.c_uint32), ("random_const", ctypes.c_void_p), ("step0", _Prog),
                ("n_pu", ctypes.c_uint32), ("pu", ctypes.c_void_p), ("step3", _Prog)]


class CommOp(ctypes.Structure):
    """zkgpu_comm_op (include/zkgpu_stark.h)"""
    _fields_ = [("peer", ctypes.c_int32), ("send", ctypes.c_int32), ("buf", ctypes.c_void_p),
                ("bytes", ctypes.c_uint64)]


EXCHANGE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(CommOp), ctypes.c_uint32)
ABORT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)


class Comm(ctypes.Structure):
    """zkgpu_comm (include/zkgpu_stark.h); abort may stay NULL"""
    _fields_ = [("rank", ctypes.c_uint32), ("world", ctypes.c_uint32), ("ctx", ctypes.c_void_p),
                ("exchange", EXCHANGE), ("abort", ABORT)]


_slib = None


def slib():
    global _slib
    if _slib is None:
        _zk_lib()  # binds the HIP runtime first (see zkgpu.lib)
        if not os.path.exists(STARK_LIB):
            raise ZkgpuError("libzkgpu_stark.so not built; run __graft_entry__.build()")
        L = ctypes.CDLL(STARK_LIB)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        for name, res, args in [
            ("zkgpu_stark_create", ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(_Info)]),
            ("zkgpu_stark_create_ex", ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(_Info), ctypes.c_uint32]),
            ("zkgpu_stark_memory_mode", ctypes.c_int, [vp]),
            ("zkgpu_stark_witness", ctypes.c_int, [vp]),
            ("zkgpu_stark_set_cm1", ctypes.c_int, [vp, vp]),
            ("zkgpu_stark_set_cm1_async", ctypes.c_int, [vp, vp]),
            ("zkgpu_stark_get_cm1", ctypes.c_int, [vp, vp]),
            ("zkgpu_stark_proof_len", u64, [vp]),
            ("zkgpu_stark_prove", ctypes.c_int, [vp, vp]),
            ("zkgpu_stark_verkey", ctypes.c_int, [vp, vp]),
            ("zkgpu_stark_publics", ctypes.c_int, [vp, vp]),
            ("zkgpu_stark_timers", ctypes.c_int, [vp, ctypes.c_char_p, u64, vp, ctypes.c_uint32]),
            ("zkgpu_stark_destroy", None, [vp]),
            ("zkgpu_stark_last_error", ctypes.c_char_p, []),
            ("zkgpu_stark_create_sharded", ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(_Info),
                                                          ctypes.POINTER(Comm)]),
            ("zkgpu_stark_memory_plan", ctypes.c_int, [ctypes.POINTER(_Info), ctypes.c_uint32,
                                                       ctypes.POINTER(u64)]),
            ("zkgpu_stark_memory_plan_ex", ctypes.c_int, [ctypes.POINTER(_Info), ctypes.c_uint32,
                                                          ctypes.POINTER(u64)]),
            ("zkgpu_comm_rccl_unique_id", ctypes.c_int, [vp]),
            ("zkgpu_comm_rccl_create", ctypes.c_int, [ctypes.POINTER(Comm), vp, ctypes.c_uint32, ctypes.c_uint32]),
            ("zkgpu_comm_rccl_destroy", None, [ctypes.POINTER(Comm)]),
            ("zkgpu_comm_host_create", ctypes.c_int, [ctypes.POINTER(Comm), ctypes.c_char_p, ctypes.c_uint32,
                                                      ctypes.c_uint32, u64]),
            ("zkgpu_comm_host_destroy", None, [ctypes.POINTER(Comm)]),
            ("zkgpu_transcript_create", vp, []),
            ("zkgpu_transcript_destroy", None, [vp]),
            ("zkgpu_transcript_put", ctypes.c_int, [vp, vp, u64]),
            ("zkgpu_transcript_get_fields1", ctypes.c_int, [vp, vp]),
            ("zkgpu_transcript_get_field", ctypes.c_int, [vp, vp]),
            ("zkgpu_transcript_get_permutations", ctypes.c_int, [vp, vp, u64, u64]),
        ]:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _slib = L
    return _slib


def _check(rc, what):
    if rc != 0:
        raise ZkgpuError("%s failed: %s" % (what, slib().zkgpu_stark_last_error().decode(errors="replace")))


class Transcript:
    """The prover's host transcript (zkgpu_transcript_*, host/starks.cpp)
    with the reference's Transcript surface (transcript.hpp:14-37): put,
    get_field, get_fields1, get_permutations.  Host code, no GPU."""

    def __init__(self):
        self._t = slib().zkgpu_transcript_create()
        if not self._t:
            raise ZkgpuError("zkgpu_transcript_create failed")

    def __del__(self):
        if getattr(self, "_t", None) and _slib is not None:
            _slib.zkgpu_transcript_destroy(self._t)
            self._t = None

    def put(self, v):
        a = np.ascontiguousarray(np.asarray(v, dtype=np.uint64).ravel())
        _check(slib().zkgpu_transcript_put(self._t, a.ctypes.data, a.size), "zkgpu_transcript_put")

    def get_fields1(self):
        o = np.zeros(1, np.uint64)
        _check(slib().zkgpu_transcript_get_fields1(self._t, o.ctypes.data), "zkgpu_transcript_get_fields1")
        return int(o[0])

    def get_field(self):
        o = np.zeros(3, np.uint64)
        _check(slib().zkgpu_transcript_get_field(self._t, o.ctypes.data), "zkgpu_transcript_get_field")
        return o

    def get_permutations(self, n, nbits):
        o = np.zeros(max(n, 1), np.uint64)
        _check(slib().zkgpu_transcript_get_permutations(self._t, o.ctypes.data, n, nbits),
               "zkgpu_transcript_get_permutations")
        return o[:n]


class RcclComm:
    """zkgpu_comm over RCCL (host/comm_rccl.hpp): rank 0 makes the id, the
    process group (any backend) carries it to the others."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        uid = np.zeros(128, np.uint8)
        if rank == 0:
            _check(slib().zkgpu_comm_rccl_unique_id(uid.ctypes.data), "zkgpu_comm_rccl_unique_id")
        if world > 1:
            t = torch.from_numpy(uid.view(np.int64).copy())
            dev = t.cuda() if dist.get_backend(group) == "nccl" else t
            dist.broadcast(dev, 0, group=group)
            uid = dev.cpu().numpy().view(np.uint8).copy()
        self.c = Comm()
        _check(slib().zkgpu_comm_rccl_create(ctypes.byref(self.c), uid.ctypes.data, world, rank),
               "zkgpu_comm_rccl_create")

    def close(self):
        slib().zkgpu_comm_rccl_destroy(ctypes.byref(self.c))


class ShmComm:
    """zkgpu_comm through host shared memory (host/comm_host.hpp): the
    processes of one machine, e.g. several ranks sharing one GPU; every rank
    passes the same name ("/...") and capacity (bytes per rank and exchange)."""

    def __init__(self, name, world, rank, capacity=1 << 30):
        self.c = Comm()
        _check(slib().zkgpu_comm_host_create(ctypes.byref(self.c), name.encode(), world, rank, capacity),
               "zkgpu_comm_host_create")

    def close(self):
        slib().zkgpu_comm_host_destroy(ctypes.byref(self.c))


class HostStagedComm:
    """zkgpu_comm over a torch.distributed group staged through host memory
    (gloo): lets two prover processes share one GPU in the tests, where RCCL
    needs one GPU per rank.  Each exchange waits for the zkgpu stream, copies
    the send slices to the host, matches the k-th send to a peer with the
    peer's k-th receive (tag k) and copies the received bytes back."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.group = group
        self.c = Comm(dist.get_rank(group), dist.get_world_size(group), None, EXCHANGE(self._exchange))

    def _exchange(self, ctx, ops, n_ops):
        try:
            import torch
            import torch.distributed as dist
            zk = _zk_lib()
            if zk.zkgpu_synchronize():
                return -1
            reqs, recvs, seq, keep = [], [], {}, []
            for k in range(n_ops):
                o = ops[k]
                tag = seq.get((o.peer, o.send), 0)
                seq[(o.peer, o.send)] = tag + 1
                t = torch.empty(o.bytes, dtype=torch.uint8)
                if o.send:
                    if zk.zkgpu_memcpy_d2h(t.data_ptr(), o.buf, o.bytes):
                        return -1
                    reqs.append(dist.isend(t, o.peer, group=self.group, tag=tag))
                else:
                    reqs.append(dist.irecv(t, o.peer, group=self.group, tag=tag))
                    recvs.append((o.buf, t))
                keep.append(t)
            for r in reqs:
                r.wait()
            for buf, t in recvs:
                if zk.zkgpu_memcpy_h2d(buf, t.data_ptr(), t.numel()):
                    return -1
            return 0
        except Exception:  # an exception must not cross the C frame
            import traceback
            traceback.print_exc()
            return -1

    def close(self):
        pass


def make_info(inst, keep):
    """zkgpu_stark_info of a SyntheticStark instance; the arrays it points
    into are appended to `keep` (they must outlive the struct)."""
    info = _Info()
    info.n_bits, info.n_bits_ext, info.n_queries = inst.n_bits, inst.n_bits_ext, inst.n_queries
    info.n_fri_steps = len(inst.fri_steps)
    for i, s in enumerate(inst.fri_steps):
        info.fri_steps[i] = s
    info.n_cm1, info.n_cm2, info.n_cm3, info.n_cm4 = inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4
    info.n_tmp, info.n_const, info.n_publics = inst.n_tmp, inst.n_const, inst.n_publics
    info.q_deg, info.l_first, info.n_k, info.seed = inst.q_deg, inst.l_first, inst.n_k, inst.seed
    rc = np.array(inst.random_cm1_cols(), np.uint32)
    zc = np.array(inst.z_ctx, np.uint32).reshape(-1)
    ev = np.array(inst.evmap, np.uint32).reshape(-1)
    rk = np.array(inst.random_const_cols(), np.uint32)
    pu = np.array(inst.pu, np.uint32).reshape(-1)
    keep += [rc, zc, ev, rk, pu]
    info.n_random_const, info.random_const = rk.size, rk.ctypes.data
    info.n_pu, info.pu = len(inst.pu), (pu.ctypes.data if pu.size else None)
    info.n_random_cols, info.random_cols = rc.size, rc.ctypes.data
    info.n_zctx, info.zctx = len(inst.z_ctx), zc.ctypes.data
    info.n_ev, info.ev = len(inst.evmap), ev.ctypes.data
    for name in ("step0", "step1", "step2", "step3prev", "step3", "step42ns", "step52ns"):
        prog = inst.programs.get(name)
        if prog is None:
            continue
        ins, opn = prog.arrays()
        ins, opn = np.ascontiguousarray(ins), np.ascontiguousarray(opn)
        keep += [ins, opn]
        setattr(info, name, _Prog(ins.ctypes.data, ins.shape[0], opn.ctypes.data, opn.shape[0],
                                  max(prog.n_tmp1, 1), max(prog.n_tmp3, 1)))
    return info


# single-GPU memory plans (include/zkgpu_stark.h ZKGPU_MEM_*)
MEM_AUTO, MEM_RESIDENT, MEM_LEAN = 0, 1, 2
MEM_NAMES = {MEM_RESIDENT: "resident", MEM_LEAN: "lean"}


def memory_plan(inst, world=0, mode=None):
    """HBM bytes per GPU of a prover of this instance (zkgpu_stark_memory_plan:
    world 0 = one GPU, W = row-sharded over W ranks; mode MEM_RESIDENT /
    MEM_LEAN for one GPU, zkgpu_stark_memory_plan_ex); no GPU needed."""
    keep = []
    info = make_info(inst, keep)
    out = ctypes.c_uint64(0)
    if mode is not None:
        if world:
            raise ValueError("memory plans other than the sharded prover's apply to one GPU (world 0)")
        _check(slib().zkgpu_stark_memory_plan_ex(ctypes.byref(info), mode, ctypes.byref(out)),
               "zkgpu_stark_memory_plan_ex")
        return out.value
    _check(slib().zkgpu_stark_memory_plan(ctypes.byref(info), world, ctypes.byref(out)), "zkgpu_stark_memory_plan")
    return out.value


class GpuStark:
    """mode: single-GPU memory plan (MEM_AUTO: resident when it fits the free
    HBM, else lean; under MEM_LEAN a proof consumes its trace, so witness()
    or set_cm1() comes before every prove)"""

    def __init__(self, inst, comm=None, mode=MEM_AUTO):
        self.inst = inst
        self._keep = []
        info = make_info(inst, self._keep)
        self._info = info
        self.h = ctypes.c_void_p()
        self.comm = comm
        if comm is None:
            _check(slib().zkgpu_stark_create_ex(ctypes.byref(self.h), ctypes.byref(info), mode),
                   "zkgpu_stark_create_ex")
        else:  # row-sharded over comm's ranks (host/sharded_starks.hpp)
            _check(slib().zkgpu_stark_create_sharded(ctypes.byref(self.h), ctypes.byref(info), ctypes.byref(comm.c)),
                   "zkgpu_stark_create_sharded")

    def witness(self):
        _check(slib().zkgpu_stark_witness(self.h), "zkgpu_stark_witness")

    def memory_mode(self):
        """"resident" / "lean" (single-GPU prover), "sharded" """
        if self.comm is not None:
            return "sharded"
        return MEM_NAMES[slib().zkgpu_stark_memory_mode(self.h)]

    def set_cm1(self, rows):
        rows = np.ascontiguousarray(rows, np.uint64)
        _check(slib().zkgpu_stark_set_cm1(self.h, rows.ctypes.data), "zkgpu_stark_set_cm1")

    def get_cm1(self):
        """cm1_n as the executor's row-major buffer (n x n_cm1)"""
        rows = np.empty((1 << self.inst.n_bits, self.inst.n_cm1), np.uint64)
        _check(slib().zkgpu_stark_get_cm1(self.h, rows.ctypes.data), "zkgpu_stark_get_cm1")
        return rows

    def set_cm1_async(self, rows):
        """queue the trace of the proof after the next one: it loads while the
        next prove() runs and is cm1_n when that returns (`rows` is kept
        referenced until then)"""
        rows = np.ascontiguousarray(rows, np.uint64)
        self._cm1_next = rows
        _check(slib().zkgpu_stark_set_cm1_async(self.h, rows.ctypes.data), "zkgpu_stark_set_cm1_async")

    def verkey(self):
        v = np.zeros(4, np.uint64)
        slib().zkgpu_stark_verkey(self.h, v.ctypes.data)
        return v

    def publics(self):
        v = np.zeros(max(self.inst.n_publics, 1), np.uint64)
        n = slib().zkgpu_stark_publics(self.h, v.ctypes.data)
        return v[:n]

    def prove_raw(self):
        n = slib().zkgpu_stark_proof_len(self.h)
        buf = np.zeros(n, np.uint64)
        _check(slib().zkgpu_stark_prove(self.h, buf.ctypes.data), "zkgpu_stark_prove")
        self._cm1_next = None  # a background cm1 load was taken by this prove
        return buf

    def prove(self):
        return self.parse(self.prove_raw())

    def timers(self):
        names = ctypes.create_string_buffer(4096)
        ms = np.zeros(64, np.float64)
        n = slib().zkgpu_stark_timers(self.h, names, len(names), ms.ctypes.data, 64)
        keys = names.value.decode().split("\n")[:n]
        return dict(zip(keys, [float(x) for x in ms[:n]]))

    def parse(self, buf):
        inst = self.inst
        q = inst.n_queries
        steps = inst.fri_steps
        pos = [0]

        def take(n, shape=None):
            a = buf[pos[0]:pos[0] + n]
            pos[0] += n
            return a.reshape(shape) if shape else a

        out = {}
        for k in ("root1", "root2", "root3", "root4"):
            out[k] = take(4)
        out["evals"] = take(3 * len(inst.evmap), (-1, 3))
        for si in range(1, len(steps)):
            width = 3 << (steps[si - 1] - steps[si])
            out["s%d_root" % si] = take(4)
            out["s%d_vals" % si] = take(q * width, (q, width))
            out["s%d_siblings" % si] = take(q * steps[si] * 4, (q, steps[si], 4))
        widths = [inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4, inst.n_const]
        tags = ["1", "2", "3", "4", "C"]
        for tag, wd in zip(tags, widths):
            out["s0_vals" + tag] = take(q * wd, (q, wd))
        for tag in tags:
            out["s0_siblings" + tag] = take(q * inst.n_bits_ext * 4, (q, inst.n_bits_ext, 4))
        out["finalPol"] = take(3 << steps[-1], (-1, 3))
        assert pos[0] == buf.size
        return to_json(out)

    def close(self):
        if self.h:
            slib().zkgpu_stark_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def to_json(proof):
    def conv(v):
        if isinstance(v, np.ndarray):
            return conv(v.tolist())
        if isinstance(v, list):
            return [conv(x) for x in v]
        return str(int(v) % P)
    out = {k: conv(proof[k]) for k in ("root1", "root2", "root3", "root4", "evals")}
    i = 1
    while "s%d_root" % i in proof:
        for k in ("root", "vals", "siblings"):
            out["s%d_%s" % (i, k)] = conv(proof["s%d_%s" % (i, k)])
        i += 1
    for tag in ("1", "2", "3", "4", "C"):
        out["s0_vals" + tag] = conv(proof["s0_vals" + tag])
    for tag in ("1", "2", "3", "4", "C"):
        out["s0_siblings" + tag] = conv(proof["s0_siblings" + tag])
    out["finalPol"] = conv(proof["finalPol"])
    return out
