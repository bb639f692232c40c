#!/usr/bin/env python3
"""Fill the on-disk code-object cache (zkevm-prover_amd/jitcache, see
csrc/zxp_jit.hip cache_dir) for the compiled expression kernels the GPU tests
and bench.py run on programs of zkEVM size: the step42ns-shaped synthetic
program (zkgpu/synthetic_bytecode.py, seed 1) at a quarter of step42ns's
opcode counts (5.3 K ops, one kernel, ~80 s of hiprtc) and at full size
(20 K ops), and the full-size step2prev / step3prev / step3 / step52ns-shaped
programs, converted like the reference's bytecode.  The full-size program
runs as segments (csrc/zxp_segment.cpp: ~8 kernels, ~30 s of hiprtc each);
hiprtc serialises threads, so the segments compile in parallel processes
(ZKGPU_ZXP_JIT_ONLY=j, one per segment).  A program's kernels depend only on
its structure, so one compile serves every proof (the reference likewise
ships its expression code compiled, chelpers/*.cpp).  No GPU needed (hiprtc
cross-compiles).

The STARK instances bench.py proves at 2^23 (the synthetic config-4
instance and the fork-9-width one of the sharded runs, bench.stark_instance)
are compiled too, one process per program: their kernels are what the
driver's bench runs, and the fork-9 ones take minutes of hiprtc that a rank
must not spend inside its timed child.

Usage: tools/jit_prebuild.py [--check] [--prune] [--quarter-only | --full-only | --only SPEC,...] [-j N]
       (--check: report cache hits only; --prune: delete the cache entries
       this run neither found nor compiled -- a hit refreshes the entry's mtime)
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd")]

import numpy as np  # noqa: E402

P = 0xFFFFFFFF00000001
SCALES = (0.25, 1.0)  # tests/test_gpu_parser.py and bench.py use the same programs
# the other zkEVM-shaped programs (tests/test_gpu_parser.py, full size)
OTHERS = ("step2prev", "step3prev", "step3", "step52ns")


def program(scale, name="step42ns"):
    import zkgpu.synthetic_bytecode as sb
    import zkgpu.parser as zp
    shape = sb.load_shape()
    ops, args = sb.generate(name, seed=1, scale=scale)
    return zp.convert(sb.PARSERS.index(name), ops, args, sb.sections(shape), shape["n_bits"], shape["n_bits_ext"])


def consts():
    rng = np.random.default_rng(0)
    return (rng.integers(0, P, (8, 3), dtype=np.uint64), rng.integers(0, P, 48, dtype=np.uint64),
            rng.integers(0, P, (2048, 3), dtype=np.uint64))


# bench.py's STARK instances at its default size (configs[3] / configs[4]),
# and the zkEVM-shaped one (zkgpu/zkevm_shaped.py; its stage programs do not
# depend on the row count, so the tests' 2^10 proof uses these kernels too)
STARKS = (("config4", False), ("fork9", True), ("zkevm", "zkevm"))
STARK_PROGS = ("step0", "step1", "step2", "step3prev", "step3", "step42ns", "step52ns")
_INSTS = {}


def stark_program(inst_name, pname):
    sys.path.insert(0, ROOT)
    if inst_name not in _INSTS:
        import bench
        _INSTS[inst_name] = bench.stark_instance(23, 1, 100, 128, dict(STARKS)[inst_name])
    return _INSTS[inst_name].programs.get(pname)


def get_program(spec):
    kind, a, b = spec.split(":")
    return program(float(b), a) if kind == "shaped" else stark_program(a, b)


def one(spec, seg):
    """child: compile segment `seg` of program `spec` (cache hit: no-op)"""
    import zkgpu
    os.environ["ZKGPU_ZXP_JIT_ONLY"] = str(seg)
    zkgpu.zxp_jit_source(get_program(spec), *consts(), rtc_check=1)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(sys.argv[2], int(sys.argv[3]))
        return
    import zkgpu
    t_start = time.time() - 1
    check = "--check" in sys.argv
    jobs = int(sys.argv[sys.argv.index("-j") + 1]) if "-j" in sys.argv else min(16, os.cpu_count() or 1)
    scales = SCALES[:1] if "--quarter-only" in sys.argv else SCALES[1:] if "--full-only" in sys.argv else SCALES
    work = [("shaped:step42ns:%g" % sc, "step42ns-shaped (seed 1, scale %g)" % sc) for sc in scales]
    if "--only" in sys.argv:  # e.g. --only shaped:step42ns:1 (A/B variants under an env switch)
        work = [(sp, sp) for sp in sys.argv[sys.argv.index("--only") + 1].split(",")]
    elif "--quarter-only" not in sys.argv:
        work += [("shaped:%s:1" % o, "%s-shaped (seed 1, scale 1)" % o) for o in OTHERS]
        if "--full-only" not in sys.argv:
            work += [("stark:%s:%s" % (i, p), "STARK %s %s" % (i, p)) for i, _ in STARKS for p in STARK_PROGS
                     if stark_program(i, p) is not None]
    # (spec, segment) units of every uncached program, compiled in parallel processes
    units, todo = [], []
    for spec, name in work:
        prog = get_program(spec)
        hit = zkgpu.zxp_jit_cached(prog, *consts())
        if check or hit:
            print("%s: %s" % (name, "cached" if hit else "NOT cached"))
            continue
        nseg = max(1, zkgpu.zxp_jit_source(prog, *consts()).count("// ---- segment "))
        units += [(spec, j) for j in range(nseg)]
        todo.append((spec, name, prog, nseg))
    t = time.time()
    running = []
    while units or running:
        while units and len(running) < jobs:
            spec, j = units.pop(0)
            running.append((spec, subprocess.Popen([sys.executable, os.path.abspath(__file__), "--one", spec, str(j)])))
        spec, pr = running[0]
        pr.wait()
        if pr.returncode:
            raise SystemExit("%s: segment compile failed (rc %d)" % (spec, pr.returncode))
        running.pop(0)
    for spec, name, prog, nseg in todo:
        assert zkgpu.zxp_jit_cached(prog, *consts()), name
        print("%s: %d kernel(s) compiled (all units: %.1f s)" % (name, nseg, time.time() - t), flush=True)
    if "--prune" in sys.argv and not check:
        d = os.path.join(ROOT, "zkevm-prover_amd", "jitcache")
        old = [f for f in os.listdir(d) if f.endswith(".co") and os.path.getmtime(os.path.join(d, f)) < t_start]
        for f in old:
            os.unlink(os.path.join(d, f))
        print("pruned %d stale cache entries" % len(old))


if __name__ == "__main__":
    main()
