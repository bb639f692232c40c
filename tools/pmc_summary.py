#!/usr/bin/env python3
"""Summarise a tools/pmc_round.sh directory into stamped profiles/<tag>_*.

Every file carries "stamps" (zkgpu/stamp.py: hashes of each kernel family's
sources and build settings at collection time); bench.py uses a profile's
counters only when the family it prices still has that stamp.

  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the default bench
  <tag>_stark_pmc.json     one config-4 proof: per kernel label launches, ms, VALU
                           wave-instructions and HBM bytes per launch, clock
  <tag>_lde_pmc.json       configs[1] LDE: the same for its pass kernels
  <tag>_s42_pmc.json       the zkEVM-shaped quotient: per pass (one launch of every segment)
  <tag>_clock.json         effective clock per label = GRBM_GUI_ACTIVE / 8 XCDs /
                           kernel time, kept only where it is <= the 2.4 GHz maximum
  <tag>_poseidon_bench.json  the isolated permutation benchmark of the shipped form

HBM bytes follow MI355X_MICROARCH.md's gfx950 correction: FETCH_SIZE and
WRITE_SIZE from separate passes, in KiB, traffic = (2 FETCH_SIZE + WRITE_SIZE) x 1024.

Usage: tools/pmc_summary.py <gpurun_out/pmc_TAG dir> <tag>
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "zkevm-prover_amd")]
from zkgpu.stamp import all_stamps  # noqa: E402

XCDS = 8
MAX_GHZ = 2.4  # MI355X_MICROARCH.md: maximum engine clock


def label(name):
    """rocprof kernel name -> the label bench.py / zkgpu_prof use"""
    base = name.split("(")[0].replace("void ", "").replace("zk::", "").strip()
    m = re.match(r"k_ntt_pass<(\d+), (\d+), (true|false)", base)
    if m:
        return "k_ntt_pass<%d,%s>" % (int(m.group(1)) + int(m.group(2)), "inv" if m.group(3) == "true" else "fwd")
    m = re.match(r"k_lde_strided<(\d+), (true|false)", base)
    if m:
        return "k_lde_%s<%s>" % ("p1" if m.group(2) == "true" else "p3", m.group(1))
    if base.startswith("zxp_jit"):
        return "zxp_jit"
    return base


def _csv(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return f[0] if f else None


def counters(d):
    """{dispatch: {"name", counter: value}}"""
    out = collections.defaultdict(dict)
    for r in csv.DictReader(open(_csv(d, "*counter_collection.csv"))):
        e = out[r["Dispatch_Id"]]
        e["name"] = r["Kernel_Name"]
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def durations(d):
    """{dispatch: seconds} from the pass's kernel trace"""
    out = {}
    f = _csv(d, "*kernel_trace.csv")
    for r in csv.DictReader(open(f)):
        out[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return out


def per_label(src, name, skip_first=0):
    """launch-summed counters per label over the SQ / FETCH / WRITE passes"""
    sq, fe, wr = (counters(os.path.join(src, "%s_%s" % (name, p))) for p in ("sq", "fetch", "write"))
    dur = durations(os.path.join(src, name + "_sq"))
    lab = collections.defaultdict(lambda: collections.defaultdict(float))
    seq = collections.defaultdict(list)  # per label, in launch order: (valu, ms)
    for disp in sorted(sq, key=int):
        e = sq[disp]
        L = lab[label(e["name"])]
        L["launches"] += 1
        L["seconds"] += dur.get(disp, 0.0)
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_WAVES", "GRBM_GUI_ACTIVE"):
            L[k] += e.get(k, 0.0)
        seq[label(e["name"])].append((e.get("SQ_INSTS_VALU", 0.0), round(dur.get(disp, 0.0) * 1e3, 4)))
    for src_pass, key in ((fe, "FETCH_SIZE"), (wr, "WRITE_SIZE")):
        for e in src_pass.values():
            lab[label(e["name"])][key] += e.get(key, 0.0)
    res = {}
    for k, L in lab.items():
        n = L["launches"]
        if not n:
            continue
        ghz = L["GRBM_GUI_ACTIVE"] / XCDS / L["seconds"] / 1e9 if L["seconds"] > 1e-4 else None
        res[k] = {"launches": int(n), "ms": round(L["seconds"] * 1e3, 4),
                  "avg_launch_ms": round(L["seconds"] * 1e3 / n, 4),
                  "valu_wave_instr_per_launch": L["SQ_INSTS_VALU"] / n,
                  "vmem_rd_wave_instr_per_launch": L["SQ_INSTS_VMEM_RD"] / n,
                  "salu_wave_instr_per_launch": L["SQ_INSTS_SALU"] / n,
                  "hbm_bytes_per_launch": (2 * L["FETCH_SIZE"] + L["WRITE_SIZE"]) * 1024.0 / n,
                  "clock_GHz": round(ghz, 3) if ghz else None,
                  "clock_valid": bool(ghz and ghz <= MAX_GHZ)}
        if n <= 64:  # the launches in order (the last ones are the timed proof's; the first may be setup)
            res[k]["launch_valu"] = [v for v, _ in seq[k]]
            res[k]["launch_ms"] = [t for _, t in seq[k]]
    return dict(sorted(res.items(), key=lambda kv: -kv[1]["ms"]))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    stamps = all_stamps()
    note = "tools/pmc_round.sh %s -> tools/pmc_summary.py" % tag
    wrote = []

    def dump(name, doc):
        doc["stamps"] = stamps
        doc["source"] = note
        with open(os.path.join(prof, "%s_%s" % (tag, name)), "w") as f:
            json.dump(doc, f, indent=1)
        wrote.append(name)

    st = _csv(os.path.join(src, "stats"), "*kernel_stats.csv")
    if st:
        shutil.copy(st, os.path.join(prof, "%s_kernel_stats.csv" % tag))
        wrote.append("kernel_stats.csv")
        b = os.path.join(src, "stats_bench.json")
        if os.path.exists(b):
            shutil.copy(b, os.path.join(prof, "%s_stats_bench.json" % tag))
    clock = {}
    if os.path.isdir(os.path.join(src, "stark_sq")):
        k = per_label(src, "stark")
        dump("stark_pmc.json", {"_doc": "one 2^23 config-4 proof (bench.py --workload stark --steps 1 --warmup 0) "
                                        "under three rocprofv3 --pmc passes; per bench label", "kernels": k})
        clock.update({x: v["clock_GHz"] for x, v in k.items() if v["clock_valid"]})
    if os.path.isdir(os.path.join(src, "lde_sq")):
        k = per_label(src, "lde")
        dump("lde_pmc.json", {"_doc": "configs[1] LDE 2^23 -> 2^24 x 100 (bench.py --workload lde --steps 2 "
                                      "--warmup 1 under three --pmc passes; the passes' launches include the warmup)",
                              "bench_labels": k})
        clock.update({x: v["clock_GHz"] for x, v in k.items() if v["clock_valid"] and x not in clock})
    if os.path.isdir(os.path.join(src, "s42_sq")):
        k = per_label(src, "s42")
        z = k.get("zxp_jit")
        if z:
            # one pass = one launch of every segment; bench.py runs 1 warmup + 2 steps
            passes = 3.0
            dump("s42_pmc.json", {
                "_doc": "the zkEVM-shaped quotient (bench.py --workload step42ns --s42-scale 1 --s42-jit, 2^24 rows, "
                        "LDS column cache as configured) under three --pmc passes; per pass = all segment launches",
                "segments": int(round(z["launches"] / passes)), "step_ms": round(z["ms"] / passes, 3),
                "hbm_bytes_per_step": z["hbm_bytes_per_launch"] * z["launches"] / passes,
                "per_step": {"SQ_INSTS_VALU": z["valu_wave_instr_per_launch"] * z["launches"] / passes,
                             "SQ_INSTS_VMEM_RD": z["vmem_rd_wave_instr_per_launch"] * z["launches"] / passes},
                "clock_GHz": z["clock_GHz"], "clock_valid": z["clock_valid"]})
    if clock:
        labels = {}
        for lab in ("k_leaves_cols", "k_merkle_level"):
            if lab in clock:
                labels[lab] = clock[lab]
        ntt = [v for x, v in clock.items() if x.startswith("k_ntt_pass")]
        if ntt:
            labels["k_ntt_pass"] = round(sum(ntt) / len(ntt), 3)
        dump("clock.json", {"_doc": "GRBM_GUI_ACTIVE / 8 XCDs / kernel time, from the SQ passes; kernels whose "
                                    "reading exceeds the %.1f GHz maximum are dropped (too short to measure)" % MAX_GHZ,
                            "kernels": clock, "labels": labels})
    pb = os.path.join(src, "poseidon_bench.txt")
    if os.path.exists(pb):
        text = open(pb).read()
        m = re.search(r"^fast \(FFT MDS \+ block dots\)\s+[\d.]+ ms\s+([\d.]+) Gperm/s", text, re.M)
        c = re.search(r"shader clock under load: ([\d.]+) GHz", text)
        dump("poseidon_bench.json", {"_doc": "tools/poseidon_bench.hip: the shipped permutation (csrc/poseidon_perm.hpp "
                                             "perm_fast) and variants, one state per thread",
                                     "fast_Gperm_s": float(m.group(1)) if m else None,
                                     "clock_GHz": float(c.group(1)) if c else None, "text": text.splitlines()})
    print("wrote", ", ".join("%s_%s" % (tag, w) for w in wrote))


if __name__ == "__main__":
    main()
