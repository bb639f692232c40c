#!/usr/bin/env python3
"""Summarise tools/job_s42pmc.sh output (gpurun_out/s42pmc) into a profile
JSON: per proof-step totals of the segment kernels of the zkEVM-sized
quotient (the last `steps` x n_seg zxp_jit dispatches of each pass), HBM
bytes per MI355X_MICROARCH.md (2 x FETCH_SIZE + WRITE_SIZE, KiB), and the
kernel-trace durations.  Usage: s42_pmc_summary.py <dir> <out.json> [steps]"""
import collections
import csv
import glob
import json
import os
import sys


def load(path):
    per = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return per, names


def main():
    src, out = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    tot = collections.defaultdict(float)
    nseg = None
    for p in ("p1", "p2", "p3", "p4"):
        f = glob.glob(os.path.join(src, p, "*counter_collection.csv"))
        if not f:
            continue
        per, names = load(f[0])
        ds = [d for d in sorted(per) if "zxp_jit" in names[d]]
        # dispatches per step: (warmup + steps) equal groups
        nseg = len(ds) // (steps + 1)
        for d in ds[-steps * nseg:]:
            for k, v in per[d].items():
                tot[k] += v / steps
    dur = []
    for f in glob.glob(os.path.join(src, "stats", "*kernel_trace.csv")):
        rows = [r for r in csv.DictReader(open(f)) if "zxp_jit" in r["Kernel_Name"]]
        rows = rows[-steps * nseg:]
        for j in range(nseg):
            ts = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows[j::nseg]]
            dur.append(round(sum(ts) / len(ts), 3))
    hbm = (2 * tot.get("FETCH_SIZE", 0) + tot.get("WRITE_SIZE", 0)) * 1024.0
    step_ms = sum(dur)
    res = {"kernel": "zxp_jit segments of the full-size step42ns-shaped quotient (2^24 rows), per proof step",
           "command": "tools/job_s42pmc.sh (bench.py --workload step42ns --s42-scale 1 --s42-jit, rocprofv3 passes)",
           "segments": nseg, "segment_ms": dur, "step_ms": round(step_ms, 3),
           "per_step": {k: v for k, v in sorted(tot.items())},
           "hbm_bytes_per_step": hbm,
           "hbm_GBs": round(hbm / (step_ms * 1e-3) / 1e9, 1) if step_ms else None,
           "valu_per_s": round(tot.get("SQ_INSTS_VALU", 0) / (step_ms * 1e-3) / 1e9, 1) if step_ms else None,
           "note": "HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 (gfx950 FETCH_SIZE half-count of wide reads, "
                   "MI355X_MICROARCH.md); FETCH_SIZE includes Infinity-Cache hits"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("segments", "segment_ms", "step_ms", "hbm_bytes_per_step", "hbm_GBs",
                                          "valu_per_s")}))


if __name__ == "__main__":
    main()
