#!/usr/bin/env python3
"""Effective clock per kernel (GHz) = GRBM_GUI_ACTIVE cycles / kernel duration
/ 8 (rocprofv3 sums the counter over the 8 XCDs' GRBM instances),
from tools/pmc_clock.sh-style rocprofv3 passes (GRBM_GUI_ACTIVE + kernel
trace).  Usage: clock_summary.py <out.json> <pass dir>...  ("labels": the
kernels bench.py's valu block reads)."""
import collections
import csv
import glob
import json
import sys

XCDS = 8


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    cyc = collections.defaultdict(float)
    dur = collections.defaultdict(float)
    for d in dirs:
        for r in csv.DictReader(open(glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0])):
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                cyc[r["Kernel_Name"]] += float(r["Counter_Value"])
        for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])):
            dur[r["Kernel_Name"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    kern = {}
    for k in cyc:
        if dur.get(k, 0) > 1e-4:
            kern[k.split("(")[0].replace("void ", "").replace("zk::", "")] = round(cyc[k] / XCDS / dur[k] / 1e9, 3)
    labels = {}
    for lab in ("k_leaves_cols", "k_merkle_level", "k_ntt_pass"):
        v = [g for k, g in kern.items() if k.startswith(lab) and (lab != "k_merkle_level" or k == lab)]
        if v:
            labels[lab] = round(sum(v) / len(v), 3)
    json.dump({"_doc": "GRBM_GUI_ACTIVE / 8 XCDs / kernel duration per kernel (tools/clock_summary.py over rocprofv3 passes "
                       "of bench.py --workload merkle / lde)", "kernels": kern, "labels": labels}, open(out, "w"),
              indent=1)
    print(labels)


if __name__ == "__main__":
    main()
