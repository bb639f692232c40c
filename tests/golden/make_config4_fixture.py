"""Generate tests/golden/config4_2p<bits>_proof.json: the oracle's proof of
bench.py's config-4 instance (bench.stark_instance: the instance the headline
bench line times) at full size, as per-field digests plus the small fields
verbatim.  tests/test_gpu_full_parity.py proves the same instance on the GPU
and compares field by field.

The oracle (oracle/stark_prover.py over oracle/*.c) is pinned by the
reference's golden proofs (tests/test_golden_proofs.py); this fixture carries
that pin to the benchmarked size.  Run in the build container (no GPU):

    python tests/golden/make_config4_fixture.py [--bits 23] [--threads 8]
    python tests/golden/make_config4_fixture.py --zkevm --bits 20

2^23 needs ~52 GB of host memory and ~30 min on 8 threads.  --zkevm: the
zkEVM-shaped instance instead (bench.stark_instance(bits, 1, 100, 128,
"zkevm"): the fork-9 widths with the five zkEVM-shaped programs, the
sharded_one_proof.fork9_zkevm_shaped workload) -> zkevm_shaped_2p<bits>_proof.json;
2^20 is the largest whose oracle run fits this container (~47 GB).
"""
import argparse
import hashlib
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd")]

SMALL = ("root1", "root2", "root3", "root4", "evals", "finalPol")


def field_digest(v):
    return hashlib.sha256(json.dumps(v, separators=(",", ":")).encode()).hexdigest()


def summarize(proof):
    """per-field sha256 of the canonical JSON, the small fields verbatim"""
    return {"fields": {k: field_digest(v) for k, v in proof.items()},
            "small": {k: proof[k] for k in SMALL if k in proof},
            "digest": field_digest(proof)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=23)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--zkevm", action="store_true")
    a = ap.parse_args()
    import bench
    from oracle import oracle as oc
    from oracle.stark_prover import OracleStark
    oc.lib().oc_set_num_threads(a.threads)
    kind = "zkevm" if a.zkevm else False
    inst = bench.stark_instance(a.bits, 1, 100, 128, kind)
    t0 = time.time()
    o = OracleStark(inst)
    o.witness()
    proof = o.prove()
    dt = time.time() - t0
    doc = {"what": ("oracle proof (oracle/stark_prover.py) of bench.stark_instance(%d, 1, 100, 128%s): %s, trace from "
                    "the instance's own witness" % (a.bits, ', "zkevm"' if a.zkevm else "",
                                                   "the zkEVM-shaped instance (fork-9 widths + the five zkEVM-shaped "
                                                   "programs)" if a.zkevm else
                                                   "the synthetic config-4 instance of bench.py's headline line")),
           "instance": {"log_n": a.bits, "blowup_bits": 1, "ncols": 100, "queries": 128, "kind": kind or "config4",
                        "n_cm": [inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4], "n_const": inst.n_const,
                        "fri_steps": list(inst.fri_steps)},
           "generated_by": "tests/golden/make_config4_fixture.py%s --bits %d --threads %d" % (
               " --zkevm" if a.zkevm else "", a.bits, a.threads),
           "oracle_seconds": round(dt, 1),
           "max_rss_GB": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 1)}
    doc.update(summarize(proof))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "%s_2p%d_proof.json" % ("zkevm_shaped" if a.zkevm else "config4", a.bits))
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print("wrote %s (%.0f s)" % (out, dt))


if __name__ == "__main__":
    main()
