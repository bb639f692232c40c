#!/usr/bin/env python3
"""Summarise rocprofv3 runs into profiles/: kernel stats + per-launch HBM traffic.

HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes (TCC slots), in KiB; on gfx950
FETCH_SIZE reports half of the bytes of a wide coalesced streaming read, so
traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.

Usage: tools/pmc_traffic.py <gpurun_out dir> <round tag, e.g. r01>
"""
import csv
import re
import json
import os
import shutil
import sys


def per_kernel(path, counter):
    agg = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        agg.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def bench_label(name):
    """rocprof kernel name -> the label bench.py / zkgpu_prof_* use."""
    base = name.split("(")[0].replace("void ", "").replace("zk::", "").strip()
    m = re.match(r"k_ntt_pass<(\d+), (\d+), (true|false)", base)
    if m:
        return "k_ntt_pass<%d,%s>" % (int(m.group(1)) + int(m.group(2)), "inv" if m.group(3) == "true" else "fwd")
    m = re.match(r"k_lde_strided<(\d+), (true|false)", base)
    if m:  # P1 = inverse, P3 = forward (ntt.hip 3-pass LDE)
        return "k_lde_%s<%s>" % ("p1" if m.group(2) == "true" else "p3", m.group(1))
    return base


def launches(path):
    n = {}
    seen = set()
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        if key not in seen:
            seen.add(key)
            n[r["Kernel_Name"]] = n.get(r["Kernel_Name"], 0) + 1
    return n


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    fetch = per_kernel(os.path.join(src, "pmc_fetch/run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "pmc_write/run_counter_collection.csv"), "WRITE_SIZE")
    out = {}
    for k in fetch:
        if k in write:
            out[k] = {"FETCH_SIZE_KiB": fetch[k], "WRITE_SIZE_KiB": write[k],
                      "hbm_bytes_per_launch": (2 * fetch[k] + write[k]) * 1024.0}
    # per bench label, launch-weighted
    cnt = launches(os.path.join(src, "pmc_write/run_counter_collection.csv"))
    by_label = {}
    for k, v in out.items():
        lab = bench_label(k)
        b = by_label.setdefault(lab, {"launches": 0, "hbm_bytes": 0.0})
        b["launches"] += cnt.get(k, 1)
        b["hbm_bytes"] += v["hbm_bytes_per_launch"] * cnt.get(k, 1)
    sq = os.path.join(src, "pmc_sqb/run_counter_collection.csv")
    valu = {}
    if os.path.exists(sq):
        vi = per_kernel(sq, "SQ_INSTS_VALU")
        vc = launches(sq)
        for k, v in vi.items():
            lab = bench_label(k)
            b = valu.setdefault(lab, [0, 0.0])
            b[0] += vc.get(k, 1)
            b[1] += v * vc.get(k, 1)
    labels = {lab: {"hbm_bytes_per_launch": b["hbm_bytes"] / b["launches"]} for lab, b in by_label.items()}
    for lab, (n, tot) in valu.items():
        labels.setdefault(lab, {})["valu_wave_instr_per_launch"] = tot / n
    meta = {"_doc": "per-launch HBM traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE half-count "
                    "correction, MI355X_MICROARCH.md HBM); separate --pmc passes of `python3 bench.py --workload lde --no-cpu "
                    "--steps 2 --warmup 1`; valu_wave_instr_per_launch = SQ_INSTS_VALU (wave instructions) from a separate SQ pass",
            "kernels": out, "bench_labels": labels}
    with open(os.path.join(dst, f"{tag}_lde_pmc.json"), "w") as f:
        json.dump(meta, f, indent=1)
    if os.path.exists(os.path.join(src, "prof/run_kernel_stats.csv")):
        shutil.copy(os.path.join(src, "prof/run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    if os.path.exists(os.path.join(src, "prof_bench.json")):
        shutil.copy(os.path.join(src, "prof_bench.json"), os.path.join(dst, f"{tag}_prof_bench.json"))
    print(json.dumps(meta, indent=1)[:2000])


if __name__ == "__main__":
    main()
