#!/usr/bin/env python3
"""Does the Merkle hashing of one commit overlap with the LDE of another on
two HIP streams?  (LDE: HBM + VALU; Poseidon leaves: VALU, ~140 GB/s.)
Times LDE(2^23 -> 2^24 x 100) and merkletree(2^24 x 100) alone, back to back
on one stream, and concurrently on two streams."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd")]

import torch  # noqa: E402
import zkgpu  # noqa: E402


def main():
    zkgpu.init(0)
    dev = torch.device("cuda", 0)
    n, ne, C = 1 << 23, 1 << 24, 100
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    trace = torch.randint(0, 2**62, (C, n), dtype=torch.int64, device=dev, generator=g)
    out = torch.empty((C, ne), dtype=torch.int64, device=dev)
    src = torch.randint(0, 2**62, (C, ne), dtype=torch.int64, device=dev, generator=g)
    nodes = torch.empty(zkgpu.merkle_num_elements(ne), dtype=torch.int64, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def lde(s):
        zkgpu.set_stream(s)
        zkgpu.extend_pol_dev(out, ne, trace, n, ne, n, C)

    def tree(s):
        zkgpu.set_stream(s)
        zkgpu.merkletree_dev(nodes, src, ne, C, ne)

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / reps * 1e3

    res = {"lde_ms": timed(lambda: lde(s1)), "tree_ms": timed(lambda: tree(s1)),
           "sequential_ms": timed(lambda: (lde(s1), tree(s1))),
           "concurrent_ms": timed(lambda: (lde(s1), tree(s2)))}
    print(res, flush=True)


if __name__ == "__main__":
    main()
