#!/usr/bin/env python3
"""Per-kernel summary of a 2^23 STARK proof under PMC (tools/gpu_job.sh starkpmc):
time, VALU wave-instructions (SQ_INSTS_VALU) and HBM
bytes/s ((2*FETCH_SIZE + WRITE_SIZE) * 1024, MI355X_MICROARCH.md gfx950
correction), from three separate --pmc passes.  Times come from the SQ pass's
kernel trace (PMC serialises kernels, so they are slightly inflated).

Usage: tools/stark_pmc.py <gpurun_out dir> <out json>
"""
import collections
import csv
import glob
import json
import sys



def counters(d):
    f = glob.glob("%s/**/*counter_collection.csv" % d, recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def times(d):
    f = glob.glob("%s/**/*kernel_trace.csv" % d, recursive=True)[0]
    t = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f)):
        t[r["Kernel_Name"]][0] += 1
        t[r["Kernel_Name"]][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return t


def main():
    src, out = sys.argv[1], sys.argv[2]
    sq, fe, wr, tt = counters(src + "/pmc_ssq"), counters(src + "/pmc_sfetch"), counters(src + "/pmc_swrite"), \
        times(src + "/pmc_ssq")
    res = {}
    for k, (n, sec) in tt.items():
        if sec <= 0:
            continue
        valu = sq.get(k, {}).get("SQ_INSTS_VALU", 0.0)
        hbm = 2 * fe.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 + wr.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        name = k.split("(")[0].replace("void ", "").replace("zk::", "")
        res[name] = {"launches": n, "ms": round(sec * 1e3, 3), "valu_wave_instr_per_launch": valu / n,
                     "valu_G_per_s": round(valu / sec / 1e9, 1),
                     "hbm_GBps": round(hbm / sec / 1e9, 1), "hbm_GB": round(hbm / 1e9, 3),
                     "hbm_bytes_per_launch": hbm / n}
    res = dict(sorted(res.items(), key=lambda kv: -kv[1]["ms"]))
    doc = {"_doc": "one 2^23 config-4 STARK proof (bench.py --workload stark --steps 1 --warmup 0) under rocprofv3 "
                   "--pmc in three passes; valu_wave_instr_per_launch = SQ_INSTS_VALU / launches (bench.py prices it against "
                   "the measured issue peak, profiles/*_instbench.json x *_valu_mix.json); "
                   "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024 bytes",
           "kernels": res}
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in list(res.items())[:25]:
        print("%-45s %s" % (k[:45], v))


if __name__ == "__main__":
    main()
