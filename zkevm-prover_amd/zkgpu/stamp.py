"""Source stamps of the kernel families a committed profile describes.

A PMC profile (profiles/*_pmc.json, *_clock.json, *_valu_mix.json, the
isolated permutation benchmark) is only evidence for the kernels it was
collected on.  tools/pmc_summary.py stamps every profile it writes with the
hash of each family's sources (and the build settings that change the
kernels); bench.py recomputes the stamps of the tree it runs from and uses a
profile's counters only when the family it needs matches -- otherwise the
figure is reported as stale and its ratios are dropped.
"""
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_COMMON = ["csrc/gl_device.hpp", "csrc/gl_rb.hpp", "csrc/zkgpu_internal.hpp", "Makefile"]
FAMILIES = {
    # the NTT pass chain of extendPol (configs[1], roofline)
    "lde": _COMMON + ["csrc/ntt.hip", "csrc/api.hip"],
    # the Merkle leaf / node kernels and the permutation (k_leaves_cols, k_merkle_level)
    "poseidon": _COMMON + ["csrc/poseidon.hip", "csrc/poseidon_perm.hpp", "csrc/poseidon_gl_sparse.h",
                           "csrc/poseidon_gl_constants.h"],
    # the run-time compiled expression kernels (quotient / FRI polynomial)
    "zxp": _COMMON + ["csrc/zxp_jit.hip", "csrc/zxp_compile.cpp", "csrc/zxp_segment.cpp", "csrc/zxp_segment.hpp",
                      "csrc/parser_convert.cpp", "csrc/parser_isa.inc", "zkgpu/synthetic_bytecode.py"],
}
# environment settings that change a family's kernels
ENV = {
    "lde": ["ZKGPU_LDE3"],
    "poseidon": [],
    # the compiler's fusion / term cap change the compiled programs (ZKGPU_ZXP_JIT,
    # interpreter vs compiled, is not one: the profiled workloads pick the
    # compiled kernels themselves, bench.py --s42-jit)
    "zxp": ["ZKGPU_ZXP_FUSE", "ZKGPU_ZXP_MAX_TERMS", "ZKGPU_ZXP_SEG_AB"],
}


def stamp(family, env=None):
    env = os.environ if env is None else env
    h = hashlib.sha256()
    for rel in FAMILIES[family]:
        h.update(rel.encode())
        with open(os.path.join(PKG, rel), "rb") as f:
            h.update(f.read())
    for k in ENV[family]:
        h.update(("%s=%s;" % (k, env.get(k, ""))).encode())
    return h.hexdigest()[:16]


def all_stamps(env=None):
    return {f: stamp(f, env) for f in FAMILIES}


def check(doc, family):
    """(ok, note) for a profile dict: ok when it carries the current stamp of
    `family`"""
    have = (doc or {}).get("stamps", {}).get(family)
    now = stamp(family)
    if have is None:
        return False, "profile has no source stamp (collected before stamping)"
    if have != now:
        return False, "profile stamp %s != current %s sources (%s)" % (have, family, now)
    return True, "stamp %s matches the %s sources" % (now, family)
