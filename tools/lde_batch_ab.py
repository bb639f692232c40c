#!/usr/bin/env python3
"""LDE time against the column batch (zkgpu_set_lde_batch_cols): 2^23 -> 2^24
rows x 256 columns, out of place and in place, 5 timed runs after one warmup
per setting (host wall time around a device synchronisation; the LDE's own
stream).  Decides the batch the lean plan may shrink to so that more of cm1's
stage-1 extension fits (host/starks.cpp choose_keep).  GPU box.

Usage: tools/lde_batch_ab.py [out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd")]


def main():
    import torch
    import zkgpu
    zkgpu.init(0)
    logn, ncols = 23, 256
    n, ne = 1 << logn, 1 << (logn + 1)
    src = torch.randint(0, 2**63 - 1, (ncols, n), dtype=torch.int64, device="cuda")
    out = torch.empty((ncols, ne), dtype=torch.int64, device="cuda")
    base = torch.empty(ncols * ne, dtype=torch.int64, device="cuda")
    res = {"what": __doc__.split("\n\n")[0], "rows": n, "cols": ncols, "batches": {}}
    ref = None
    for batch in (0, 96, 64, 48, 32, 16):
        zkgpu.set_lde_batch_cols(batch)
        times = {}
        for mode in ("out_of_place", "in_place"):
            ts = []
            for rep in range(6):
                if mode == "in_place":
                    base[:ncols * n].copy_(src.reshape(-1))
                torch.cuda.synchronize()
                t = time.perf_counter()
                if mode == "in_place":
                    zkgpu.extend_pol_inplace_dev(base, ne, n, ncols)
                else:
                    zkgpu.extend_pol_dev(out, ne, src, n, ne, n, ncols)
                torch.cuda.synchronize()
                if rep:
                    ts.append((time.perf_counter() - t) * 1e3)
            times[mode] = {"ms_median": sorted(ts)[len(ts) // 2], "ms": [round(x, 3) for x in ts]}
        h = int(out[ncols - 1, 12345].item()) ^ int(base[(ncols - 1) * ne + 12345].item())
        if ref is None:
            ref = h
        times["same_result"] = h == ref and torch.equal(out, base.reshape(ncols, ne))
        res["batches"][str(batch or "default (2^31 / n_ext = 128)")] = times
        print(batch, json.dumps(times), flush=True)
    zkgpu.set_lde_batch_cols(0)
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
