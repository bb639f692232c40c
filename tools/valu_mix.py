#!/usr/bin/env python3
"""Static VALU instruction mix per kernel of the shipped gfx950 code object.

bench.py prices an integer-VALU-bound kernel against an issue peak built from
the measured per-instruction issue costs (tools/instbench.hip,
profiles/*_instbench.json) weighted by the kernel's VALU instruction mix.  The
mix comes from the disassembly of lib/libzkgpu.so: every `v_*` instruction of
the kernel's body, `_e32/_e64/_dpp/_sdwa` encodings folded together.  Static
counts weight each instruction once; the hot kernels this is used for
(Poseidon leaves / levels, NTT passes) are fully unrolled straight-line
bodies, so the static mix is their dynamic mix up to the prologue.

Usage: tools/valu_mix.py <tag, e.g. r02> [kernel substrings ...]
"""
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
LIB = os.path.join(ROOT, "zkevm-prover_amd", "lib", "libzkgpu.so")

# demangled-name prefixes -> bench.py / zkgpu_prof labels
LABELS = [
    (r"^zk::k_leaves_cols\b", "k_leaves_cols"),
    (r"^zk::k_merkle_level\(", "k_merkle_level"),
    (r"^zk::k_merkle_level_lp\b", "k_merkle_level_lp"),
    (r"^void zk::k_ntt_pass<(\d+), (\d+), (true|false), (true|false)>", None),
]


def label(demangled):
    for pat, lab in LABELS:
        m = re.match(pat, demangled)
        if m and lab:
            return lab
        if m:
            return "k_ntt_pass<%d,%s>" % (int(m.group(1)) + int(m.group(2)), "inv" if m.group(3) == "true" else "fwd")
    return None


def kernels(lib):
    with tempfile.TemporaryDirectory() as td:
        dst = os.path.join(td, "lib.so")
        with open(lib, "rb") as f, open(dst, "wb") as g:
            g.write(f.read())
        subprocess.run([OBJDUMP, "--offloading", dst], cwd=td, check=True, capture_output=True)
        out = {}
        for obj in sorted(glob.glob(os.path.join(td, "*gfx950"))):
            txt = subprocess.run([OBJDUMP, "-d", "-C", obj], check=True, capture_output=True, text=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
                if m:
                    cur = out.setdefault(m.group(1), collections.Counter())
                    continue
                m = re.match(r"^\s+(v_[a-z0-9_]+)", line)
                if m and cur is not None:
                    ins = re.sub(r"_(e32|e64|dpp|sdwa)$", "", m.group(1))
                    cur[ins] += 1
        return out


def main():
    tag = sys.argv[1]
    ks = kernels(LIB)
    res = {}
    for name, hist in ks.items():
        lab = label(name)
        if not lab or not hist:
            continue
        r = res.setdefault(lab, {"histogram": collections.Counter(), "symbols": []})
        r["histogram"].update(hist)
        r["symbols"].append(name)
    for r in res.values():
        r["histogram"] = dict(r["histogram"].most_common())
        r["valu_total"] = sum(r["histogram"].values())
    sys.path.insert(0, os.path.join(ROOT, "zkevm-prover_amd"))
    from zkgpu.stamp import all_stamps
    doc = {"_doc": "static VALU instruction histogram per kernel label of lib/libzkgpu.so (tools/valu_mix.py); "
                   "bench.py weights the measured issue costs (profiles/*_instbench.json) with it",
           "kernels": res, "stamps": all_stamps()}
    path = os.path.join(ROOT, "profiles", "%s_valu_mix.json" % tag)
    json.dump(doc, open(path, "w"), indent=1)
    for lab, r in res.items():
        top = list(r["histogram"].items())[:8]
        print("%-22s %6d VALU  %s" % (lab, r["valu_total"], top))


if __name__ == "__main__":
    main()
