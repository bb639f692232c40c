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

Usage: tools/jit_prebuild.py [--check] [--prune] [--quarter-only | --full-only] [-j N]
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


def one(scale, seg, name):
    """child: compile segment `seg` of program `name` at `scale` (cache hit: no-op)"""
    import zkgpu
    os.environ["ZKGPU_ZXP_JIT_ONLY"] = str(seg)
    zkgpu.zxp_jit_source(program(scale, name), *consts(), rtc_check=1)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(float(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
        return
    import zkgpu
    t_start = time.time() - 1
    check = "--check" in sys.argv
    jobs = int(sys.argv[sys.argv.index("-j") + 1]) if "-j" in sys.argv else min(16, os.cpu_count() or 1)
    scales = SCALES[:1] if "--quarter-only" in sys.argv else SCALES[1:] if "--full-only" in sys.argv else SCALES
    work = [("step42ns", sc) for sc in scales]
    if "--quarter-only" not in sys.argv:
        work += [(o, 1.0) for o in OTHERS]
    for pname, scale in work:
        name = "%s-shaped (seed 1, scale %g)" % (pname, scale)
        prog = program(scale, pname)
        hit = zkgpu.zxp_jit_cached(prog, *consts())
        if check or hit:
            print("%s: %s" % (name, "cached" if hit else "NOT cached"))
            continue
        nseg = max(1, zkgpu.zxp_jit_source(prog, *consts()).count("// ---- segment "))
        t = time.time()
        pending = list(range(nseg))
        running = []
        while pending or running:
            while pending and len(running) < jobs:
                j = pending.pop(0)
                running.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--one", str(scale),
                                                 str(j), pname]))
            running[0].wait()
            if running[0].returncode:
                raise SystemExit("%s: segment compile failed (rc %d)" % (name, running[0].returncode))
            running.pop(0)
        assert zkgpu.zxp_jit_cached(prog, *consts()), name
        print("%s: %d kernel(s) compiled in %.1f s" % (name, nseg, time.time() - t), flush=True)
    if "--prune" in sys.argv and not check:
        d = os.path.join(ROOT, "zkevm-prover_amd", "jitcache")
        old = [f for f in os.listdir(d) if f.endswith(".co") and os.path.getmtime(os.path.join(d, f)) < t_start]
        for f in old:
            os.unlink(os.path.join(d, f))
        print("pruned %d stale cache entries" % len(old))


if __name__ == "__main__":
    main()
