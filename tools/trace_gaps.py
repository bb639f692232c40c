"""Idle gaps of the GPU inside the last timed proof of a rocprofv3 kernel
trace (tools/gpu_trace.sh): the window is the last `ms_per_step` of the
trace (from the bench line written beside it) up to the proof's last
dispatch, every gap between the union of kernel intervals is listed with the
dispatches either side.

    python3 tools/trace_gaps.py gpurun_out/trace_c4 gpurun_out/trace_c4_bench.json [top]
"""
import csv
import glob
import json
import os
import sys


def main():
    d, bench = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:44],
                 int(r["Grid_Size_X"])) for r in csv.DictReader(open(f)))
    # the bench's max-over-ranks scalar (an 8-byte upload and read-back after
    # the timed region) is not part of the proof
    while len(ks) > 1 and "copyBuffer" in ks[-1][2] and ks[-1][3] <= 512 and ks[-1][0] - ks[-2][1] > 100000:
        ks.pop()
    ks = [k[:3] for k in ks]
    line = [json.loads(x) for x in open(bench) if x.startswith("{")][-1]
    ms = line["ms_per_step"]
    t1 = max(e for _, e, _ in ks)
    t0 = t1 - ms * 1e6
    a = next(i for i, k in enumerate(ks) if k[0] >= t0)
    busy, end, gaps = 0, ks[a][0], []
    for i in range(a, len(ks)):
        s, e, _ = ks[i]
        if s > end:
            gaps.append(((s - end) / 1e3, ks[i - 1][2], ks[i][2], i))
        busy += max(0, e - max(s, end))
        end = max(end, e)
    span = (end - ks[a][0]) / 1e6
    print("window %.2f ms (ms_per_step %.2f), %d dispatches, busy %.2f ms, idle %.2f ms in %d gaps"
          % (span, ms, len(ks) - a, busy / 1e6, span - busy / 1e6, len(gaps)))
    for g in sorted(gaps, reverse=True)[:top]:
        print("%8.0f us  after %-44s before %-44s #%d" % g)


if __name__ == "__main__":
    main()
