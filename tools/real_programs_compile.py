#!/usr/bin/env python3
"""The reference's own zkEVM programs through the GPU expression compiler
(VERDICT r5 "next" 6; build container, no GPU).

For each of the five fork-9 Steps programs (step2prev, step3prev, step3,
step42ns, step52ns: `op*` / `args*` of
src/starkpil/zkevm/chelpers/zkevm.chelpers.<step>.parser.hpp, read from
/root/reference at run time -- nothing of them is stored) and, beside each,
the synthetic program of the same shape that the GPU tests and bench.py run
(zkgpu/synthetic_bytecode.py, seed 1, from tests/golden/zkevm_bytecode_shape.json):
  bytecode -> zkgpu_parser_convert (the product converter, the fork-9 memory
  map) -> zkgpu_zxp_compile (host compiler) -> the run-time kernel source
  (straight-line HIP, cut into segments) -> hiprtc for gfx950, one process per
  segment;
and from each segment's code object (its AMDHSA metadata and disassembly):
VGPRs, VGPR spills, SGPRs, scratch and LDS bytes per lane / workgroup, the
occupancy it was compiled for, and its instruction counts (all, VALU, vector
memory, LDS).  Output: profiles/r06_real_programs_compile.json.

The real programs compile into a private cache (ZKGPU_JIT_CACHE under /tmp):
their kernels are not shipped, only these figures.

Usage: tools/real_programs_compile.py [-j N] [--only step42ns,...] [out.json]
"""
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd"), os.path.join(ROOT, "tools")]

LLVM = "/opt/rocm/lib/llvm/bin"
PARSERS = ("step2prev", "step3prev", "step3", "step42ns", "step52ns")
P = 0xFFFFFFFF00000001


def program(kind, name):
    import zkgpu.parser as zp
    import zkgpu.synthetic_bytecode as sb
    shape = sb.load_shape()
    if kind == "real":
        import parser_isa
        ops, args = parser_isa.load_bytecode(name)
    else:
        ops, args = sb.generate(name, seed=1, scale=1.0)
    prog = zp.convert(sb.PARSERS.index(name), ops, args, sb.sections(shape), shape["n_bits"], shape["n_bits_ext"])
    return prog, int(len(ops))


def consts():
    import numpy as np
    rng = np.random.default_rng(0)
    return (rng.integers(0, P, (8, 3), dtype=np.uint64), rng.integers(0, P, 48, dtype=np.uint64),
            rng.integers(0, P, (2048, 3), dtype=np.uint64))


def child(kind, name, seg, dump):
    """one segment: compile (or take from the cache) and dump its code object"""
    import zkgpu
    os.environ["ZKGPU_ZXP_JIT_ONLY"] = str(seg)
    os.environ["ZKGPU_ZXP_JIT_DUMP"] = dump
    prog, _ = program(kind, name)
    zkgpu.zxp_jit_source(prog, *consts(), rtc_check=2)


def metadata(co):
    """AMDHSA kernel metadata of a code object (llvm-readelf --notes)"""
    txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True, text=True).stdout
    out = {}
    for key in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "sgpr_spill_count", "group_segment_fixed_size",
                "private_segment_fixed_size", "agpr_count"):
        m = re.search(r"\.%s:\s+(\d+)" % key, txt)
        if m:
            out[key] = int(m.group(1))
    return out


def instructions(co):
    """instruction counts of the disassembly"""
    txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], capture_output=True,
                         text=True).stdout
    n = valu = vmem = lds = smem = 0
    for line in txt.splitlines():
        m = re.match(r"\s+([sv]_\w+|global_\w+|buffer_\w+|ds_\w+|flat_\w+|scratch_\w+)", line)
        if not m:
            continue
        op = m.group(1)
        n += 1
        if op.startswith("v_"):
            valu += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            vmem += 1
        elif op.startswith("ds_"):
            lds += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            smem += 1
    return {"instructions": n, "valu": valu, "vmem": vmem, "lds": lds, "smem_loads": smem}


def waves_per_simd(vgprs):
    """occupancy the register count allows (512 VGPRs per SIMD lane, granule 8)"""
    v = max(8, (vgprs + 7) // 8 * 8)
    return min(8, 512 // v)


def main():
    jobs = int(sys.argv[sys.argv.index("-j") + 1]) if "-j" in sys.argv else min(8, os.cpu_count() or 1)
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else PARSERS
    outp = [a for a in sys.argv[1:] if a.endswith(".json")]
    out_path = outp[0] if outp else os.path.join(ROOT, "profiles", "r06_real_programs_compile.json")
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5])
        return
    import zkgpu
    tmp = tempfile.mkdtemp(prefix="zkgpu_realprog_")
    real_cache = os.path.join(tempfile.gettempdir(), "zkgpu_real_jitcache")
    os.makedirs(real_cache, exist_ok=True)
    doc = {"what": __doc__.split("\n\n")[0].strip(), "generated_by": "tools/real_programs_compile.py",
           "programs": {}}
    for name in only:
        for kind in ("real", "synthetic"):
            env = dict(os.environ)
            if kind == "real":
                env["ZKGPU_JIT_CACHE"] = real_cache
            prog, n_ops = program(kind, name)
            ins, opn = prog.arrays()
            os.environ["ZKGPU_JIT_CACHE"] = env.get("ZKGPU_JIT_CACHE", "")
            if kind != "real":
                os.environ.pop("ZKGPU_JIT_CACHE", None)
            src = zkgpu.zxp_jit_source(prog, *consts())
            nseg = max(1, src.count("// ---- segment "))
            t0 = time.time()
            running, segs = [], list(range(nseg))
            while segs or running:
                while segs and len(running) < jobs:
                    j = segs.pop(0)
                    dump = os.path.join(tmp, "%s_%s.co" % (kind, name))
                    running.append((j, subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", kind,
                                                         name, str(j), dump], env=env)))
                j, pr = running.pop(0)
                if pr.wait():
                    raise SystemExit("%s %s segment %d: compile failed" % (kind, name, j))
            dt = time.time() - t0
            rec = {"bytecode_ops": n_ops, "zxp_instructions": int(ins.shape[0]), "zxp_operands": int(opn.shape[0]),
                   "tmp1": int(prog.n_tmp1), "tmp3": int(prog.n_tmp3), "segments": nseg,
                   "source_bytes": len(src), "compile_s_wall": round(dt, 1), "segment": []}
            for j in range(nseg):
                co = os.path.join(tmp, "%s_%s.co" % (kind, name)) + ("." + str(j) if nseg > 1 else "")
                m = metadata(co)
                m.update(instructions(co))
                m["waves_per_simd_by_vgprs"] = waves_per_simd(m.get("vgpr_count", 0))
                m["code_bytes"] = os.path.getsize(co)
                rec["segment"].append(m)
            segs_ = rec["segment"]
            rec["total"] = {k: sum(s.get(k, 0) for s in segs_)
                            for k in ("instructions", "valu", "vmem", "lds", "vgpr_spill_count", "code_bytes")}
            rec["max_vgprs"] = max(s.get("vgpr_count", 0) for s in segs_)
            rec["max_scratch_bytes_per_lane"] = max(s.get("private_segment_fixed_size", 0) for s in segs_)
            doc["programs"].setdefault(name, {})[kind] = rec
            print("%-9s %-9s ops %6d zxp %6d segs %2d maxVGPR %3d spills %5d scratch %5d VALU %7d vmem %6d (%.0f s)"
                  % (name, kind, n_ops, ins.shape[0], nseg, rec["max_vgprs"], rec["total"]["vgpr_spill_count"],
                     rec["max_scratch_bytes_per_lane"], rec["total"]["valu"], rec["total"]["vmem"], dt), flush=True)
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print("wrote", out_path)


if __name__ == "__main__":
    main()
