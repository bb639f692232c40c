#!/usr/bin/env python3
"""Sum tools/pmc_s42_stall.sh passes over the zxp_jit launches (one step)."""
import collections, csv, glob, os, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/s42_stall"
tot = collections.defaultdict(float)
for f in sorted(glob.glob(os.path.join(d, "p*", "p_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "zxp_jit" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for f in sorted(glob.glob(os.path.join(d, "p1", "p_kernel_trace.csv"))):
    ms = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in csv.DictReader(open(f))
             if "zxp_jit" in r["Kernel_Name"])
    print("zxp_jit ms %.2f" % ms)
for k in sorted(tot):
    print("%-24s %.4g" % (k, tot[k]))
wc = tot.get("SQ_WAVE_CYCLES", 0)
if wc:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
              "SQ_IFETCH", "SQ_WAIT_INST_LDS"):
        if k in tot:
            print("%-24s / wave cycles = %.3f" % (k, tot[k] / wc))
