#!/usr/bin/env python3
"""Summarise tools/pmc_northstar.sh: per kernel of the north-star proof
(the dispatches after the witness: the last k_rand_cols and the step1
program), device
time, VALU wave-instructions against the mix-weighted issue peak (978 G
wave-instr/s) and HBM traffic = (2 FETCH_SIZE +
WRITE_SIZE) x 1 KiB (MI355X_MICROARCH.md gfx950 correction) against 8 TB/s.
The expression kernels (all named zxp_jit) are told apart by their order:
the proof runs step2, step3prev, step3, step42ns, step52ns (their segments
consecutively).

Usage: tools/pmc_northstar_sum.py gpurun_out/nspmc [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys

ISSUE_PEAK = 978e9
HBM_PEAK = 8e12


def load(d, name):
    f = glob.glob(os.path.join(d, name, "*counter_collection.csv"))[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": r["Kernel_Name"].split("(")[0], "t": (int(r["End_Timestamp"]) -
                                                                              int(r["Start_Timestamp"])) * 1e-9})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


def main():
    d = sys.argv[1]
    sq, fe, wr = load(d, "sq"), load(d, "fetch"), load(d, "write")
    ids = list(sq)
    # the witness: k_rand_cols, then the step1 program (the executor stand-in)
    start = max(i for i in ids if "k_rand_cols" in sq[i]["name"]) + 1
    while sq[start]["name"] != "zxp_jit":
        start += 1
    while sq[start]["name"] == "zxp_jit":
        start += 1
    proof = [i for i in ids if i >= start]
    # expression-kernel groups in proof order (consecutive zxp_jit runs)
    groups, prev = [], None
    for i in proof:
        if sq[i]["name"] == "zxp_jit":
            if prev != "zxp_jit":
                groups.append([])
            groups[-1].append(i)
        prev = sq[i]["name"]
    names = ["step2", "step3prev", "step3", "step42ns", "step52ns"]
    label = {}
    for g, ds in enumerate(groups):
        for i in ds:
            label[i] = "zxp_jit:" + (names[g] if g < len(names) else "group%d" % g)
    agg = collections.OrderedDict()
    for i in proof:
        name = label.get(i, sq[i]["name"].replace("zk::", "").replace("void ", ""))
        a = agg.setdefault(name, {"launches": 0, "s": 0.0, "valu": 0.0, "fetch_kib": 0.0, "write_kib": 0.0})
        a["launches"] += 1
        a["s"] += sq[i]["t"]
        a["valu"] += sq[i].get("SQ_INSTS_VALU", 0.0)
        a["fetch_kib"] += fe.get(i, {}).get("FETCH_SIZE", 0.0)
        a["write_kib"] += wr.get(i, {}).get("WRITE_SIZE", 0.0)
    out = {"what": __doc__.split("\n\n")[0], "proof_dispatches": len(proof), "kernels": {}}
    tot = sum(a["s"] for a in agg.values())
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["s"]):
        hbm = (2 * a["fetch_kib"] + a["write_kib"]) * 1024.0
        out["kernels"][name] = {"launches": a["launches"], "ms": round(a["s"] * 1e3, 3),
                                "share": round(a["s"] / tot, 4),
                                "valu_frac": round(a["valu"] / a["s"] / ISSUE_PEAK, 3) if a["s"] else None,
                                "hbm_GB": round(hbm / 1e9, 2),
                                "hbm_TBps": round(hbm / a["s"] / 1e12, 2) if a["s"] else None,
                                "hbm_frac": round(hbm / a["s"] / HBM_PEAK, 3) if a["s"] else None}
    out["device_ms"] = round(tot * 1e3, 2)
    for name, k in list(out["kernels"].items())[:16]:
        print("%-32s %3d x %9.2f ms %5.1f %%  valu %5.2f  hbm %7.1f GB %5.2f TB/s" % (
            name[:32], k["launches"], k["ms"], 100 * k["share"], k["valu_frac"] or 0, k["hbm_GB"], k["hbm_TBps"] or 0))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
