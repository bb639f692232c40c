#!/usr/bin/env python3
"""Fill the on-disk code-object cache (zkevm-prover_amd/jitcache, see
csrc/zxp_jit.hip cache_dir) for the compiled expression kernels the GPU tests
and bench.py run on programs of zkEVM size: the step42ns-shaped synthetic
program (zkgpu/synthetic_bytecode.py, seed 1) at a quarter of step42ns's
opcode counts (5.3 K ops, ~80 s of hiprtc), converted like the reference's
bytecode; --full also compiles the full-size 20 K-op program (~10 min, not
part of build()).  A program's kernel depends only on its structure, so
one compile serves every proof (the reference likewise ships its expression
code compiled, chelpers/*.cpp).  No GPU needed (hiprtc cross-compiles).

Usage: tools/jit_prebuild.py [--check] [--full]   (--check: report cache hits only)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd")]

import numpy as np  # noqa: E402

P = 0xFFFFFFFF00000001
JIT_SCALE = 0.25  # tests/test_gpu_parser.py uses the same program


def programs(full=False):
    import zkgpu.parser as zp
    import zkgpu.synthetic_bytecode as sb
    shape = sb.load_shape()
    for scale in (JIT_SCALE, 1.0) if full else (JIT_SCALE,):
        ops, args = sb.generate("step42ns", seed=1, scale=scale)
        prog = zp.convert(zp.STEP42NS, ops, args, sb.sections(shape), shape["n_bits"], shape["n_bits_ext"])
        yield "step42ns-shaped (seed 1, scale %g)" % scale, prog


def main():
    import zkgpu
    check = "--check" in sys.argv
    rng = np.random.default_rng(0)
    ch = rng.integers(0, P, (8, 3), dtype=np.uint64)
    pub = rng.integers(0, P, 48, dtype=np.uint64)
    ev = rng.integers(0, P, (2048, 3), dtype=np.uint64)
    for name, prog in programs("--full" in sys.argv):
        t = time.time()
        if check:
            hit = zkgpu.zxp_jit_cached(prog, ch, pub, ev)
            print("%s: %s" % (name, "cached" if hit else "NOT cached"))
            continue
        if zkgpu.zxp_jit_cached(prog, ch, pub, ev):
            print("%s: cached" % name)
            continue
        zkgpu.zxp_jit_source(prog, ch, pub, ev, rtc_check=1)
        print("%s: compiled in %.1f s" % (name, time.time() - t), flush=True)


if __name__ == "__main__":
    main()
