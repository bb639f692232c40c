#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X STARK hot path.

Workload (BASELINE.json configs[1]): the Goldilocks LDE of a 2^23-row trace to
2^24 rows (blowup 2, coset shift 7), column-major in HBM, C = 100 committed
columns per GPU -- NTT_Goldilocks::extendPol as called at starks.cpp:53.
One "step" = one LDE of the whole per-GPU trace, inputs already resident in
HBM.  Multi-GPU: columns are independent, so every rank extends its own 100
columns with no data-path collective (weak scaling); the barrier + max over
ranks of the timed region stay.

value = LDE output elements produced by all ranks / second (Gelem/s).
roofline = the dominant kernel (largest device time in the timed region),
measured live with HIP events on the launch stream (zkgpu_prof_*), against
8 TB/s; its algorithmic bytes per launch = every input element read once +
every output element written once.
cpu_baseline = the oracle's OpenMP LDE (oracle/ntt.c, a port of the
reference algorithm) on a bounded sample (rank 0, N = 1 only).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--ncols C] [--log-n L]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zkevm-prover_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "batch-proof STARK sec (2^23 trace) + Goldilocks NTT Gelem/s at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ncols", type=int, default=100)
    ap.add_argument("--log-n", type=int, default=23)
    ap.add_argument("--blowup-bits", type=int, default=1)
    ap.add_argument("--cpu-sample-cols", type=int, default=int(os.environ.get("ZKGPU_CPU_SAMPLE_COLS", "4")))
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--workload", choices=["lde", "merkle", "stark", "commit", "stark-sharded"], default="lde",
                    help="lde = configs[1] (headline); merkle = configs[2] (2^23 x 100 Poseidon tree); "
                         "stark = configs[3] (full synthetic STARK proof, 2^23 trace); "
                         "commit = configs[4] (one trace column-sharded over the ranks: LDE + all-to-all + "
                         "subtree Merkle + root, strong scaling)")
    ap.add_argument("--queries", type=int, default=128)
    ap.add_argument("--cpu-sample-bits", type=int, default=int(os.environ.get("ZKGPU_CPU_SAMPLE_BITS", "16")))
    return ap.parse_args()


def cpu_baseline(log_n, blow, ncols_sample):
    """Oracle LDE (OpenMP) on a bounded sample: 2^log_n -> 2^(log_n+blow) x ncols_sample."""
    import numpy as np
    from oracle import oracle as oc
    oc.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    oc.lib().oc_set_num_threads(threads)
    rng = np.random.default_rng(0x5EED)
    x = rng.integers(0, 2**63, size=(1 << log_n, ncols_sample), dtype=np.uint64)
    t0 = time.perf_counter()
    oc.extend_pol(x, 1 << (log_n + blow))
    dt = time.perf_counter() - t0
    out_elems = (1 << (log_n + blow)) * ncols_sample
    return {"value": out_elems / dt / 1e9, "unit": "Gelem/s", "cores": threads, "kind": "port",
            "sample": "oracle extendPol 2^%d->2^%d x %d cols, %.1f s, %d threads (%s)"
                      % (log_n, log_n + blow, ncols_sample, dt, threads, _cpu_model())}


def cpu_baseline_merkle(log_n, ncols):
    """Oracle merkletree (OpenMP) on a bounded sample of the same shape (fewer rows)."""
    import numpy as np
    from oracle import oracle as oc
    oc.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    oc.lib().oc_set_num_threads(threads)
    rows = 1 << min(log_n, 16)
    rng = np.random.default_rng(0x5EED)
    x = rng.integers(0, 2**63, size=(rows, ncols), dtype=np.uint64)
    t0 = time.perf_counter()
    oc.merkletree(x)
    dt = time.perf_counter() - t0
    return {"value": rows * ncols / dt / 1e9, "unit": "Gelem/s", "cores": threads, "kind": "port",
            "sample": "oracle merkletree 2^%d rows x %d cols, %.1f s, %d threads (%s)"
                      % (min(log_n, 16), ncols, dt, threads, _cpu_model())}


def cpu_baseline_commit(log_n, blow, ncols, sample_bits):
    """Oracle LDE + merkletree (OpenMP) of the same column count at 2^sample_bits rows."""
    import numpy as np
    from oracle import oracle as oc
    oc.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    oc.lib().oc_set_num_threads(threads)
    rows = 1 << min(log_n, sample_bits)
    rng = np.random.default_rng(0x5EED)
    x = rng.integers(0, 2**63, size=(rows, ncols), dtype=np.uint64)
    t0 = time.perf_counter()
    oc.merkletree(oc.extend_pol(x, rows << blow))
    dt = time.perf_counter() - t0
    return {"value": (rows << blow) * ncols / dt / 1e9, "unit": "Gelem/s", "cores": threads, "kind": "port",
            "sample": "oracle extendPol + merkletree 2^%d rows x %d cols, %.1f s, %d threads (%s)"
                      % (min(log_n, sample_bits), ncols, dt, threads, _cpu_model())}


def stark_instance(log_n, blow, ncols, n_queries):
    """cm1/cm2/cm3 = ncols/24/24, 30 constants, qDeg 2,
    FRI steps [nBitsExt, -4, ..., 5], n_queries queries (synthetic AIR)."""
    from zkgpu.synthetic import SyntheticStark
    nbe = log_n + blow
    steps = [nbe]
    while steps[-1] - 4 >= 5:
        steps.append(steps[-1] - 4)
    if steps[-1] > 5:
        steps.append(5)
    # cm1 = 3t constrained triples + free columns + 3 lookup columns (A, B, C);
    # cm2 = 6 h groups (18) + plookup h1/h2 (3+3+1+1) = 26, cm3 = 18 + 2 plookup Z = 24,
    # constants = 26 K + L_first + 3 tables = 30
    t = (ncols - 3) // 3
    return SyntheticStark(n_bits=log_n, blowup_bits=blow, t=t, n_free=ncols - 3 - 3 * t, m=6, n_k=26,
                          n_queries=n_queries, fri_steps=steps, n_lookups=2)


def cpu_baseline_stark(sample_bits, log_n, blow, ncols, n_queries):
    """Oracle STARK prover (C/OpenMP kernels + numpy driver) on a bounded sample:
    the same instance shape at 2^sample_bits rows."""
    from oracle import oracle as oc
    from oracle.stark_prover import OracleStark
    oc.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    oc.lib().oc_set_num_threads(threads)
    inst = stark_instance(sample_bits, blow, ncols, n_queries)
    o = OracleStark(inst)
    o.witness()
    t0 = time.perf_counter()
    o.prove()
    dt = time.perf_counter() - t0
    scale = (1 << (log_n - sample_bits)) * (log_n + blow) / (sample_bits + blow)
    return {"value": round(dt, 3), "unit": "s/proof (2^%d sample)" % sample_bits, "cores": threads, "kind": "port",
            "extrapolated_full_s": round(dt * scale, 1),
            "sample": "oracle genProof of the config-4 instance shape at 2^%d rows (%d cm1 cols, %d queries), "
                      "%.1f s, %d threads (%s); extrapolated_full_s scales by N log N to 2^%d"
                      % (sample_bits, ncols, n_queries, dt, threads, _cpu_model(), log_n)}


VALU_PEAK_WAVE_INSTR_S = 256 * 4 * 2.4e9 / 4  # 256 CUs x 4 SIMDs, one wave64 VALU op per 4 clk @ 2.4 GHz


def _profile_order(path):
    """Natural order of profiles/rNN_vM_* names (r01_v10 after r01_v9); the
    newest summary wins.  File mtimes are not used: a fresh checkout or a
    gpurun snapshot gives every file the same one."""
    import re
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]


def pmc_for(kernel, args, avg_ms):
    """HBM traffic and VALU issue for the dominant kernel from the committed
    PMC summaries (separate rocprofv3 --pmc passes of this same command):
    profiles/*_pmc_traffic.json (tools/pmc_traffic.py) for the default LDE
    workload, profiles/*_stark_pmc.json (tools/stark_pmc.py) for the 2^23
    STARK proof.  Returns (traffic bytes per launch or None, valu dict or None)."""
    import glob
    if args.log_n != 23 or args.ncols != 100 or args.blowup_bits != 1:
        return None, None
    if args.workload == "stark":
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_stark_pmc.json")), key=_profile_order)
        for f in reversed(files):
            try:
                ks = json.load(open(f)).get("kernels", {})
            except (OSError, ValueError):
                continue
            lab = ks.get(kernel)
            if not lab or not lab.get("launches"):
                continue
            valu = {"kernel": kernel, "achieved": round(lab["valu_frac"] * VALU_PEAK_WAVE_INSTR_S / 1e9, 1),
                    "peak": VALU_PEAK_WAVE_INSTR_S / 1e9, "unit": "G wave-instr/s",
                    "frac": lab["valu_frac"], "source": os.path.basename(f),
                    "note": ("SQ_INSTS_VALU x 4 clk / (kernel time x 1024 SIMDs) over the kernel's launches "
                             "in one 2^23 proof; > 1 means part of the stream issues faster than "
                             "4 clk per wave64 op, i.e. VALU issue is saturated")}
            return lab["hbm_GB"] * 1e9 / lab["launches"], valu
        return None, None
    if args.workload != "lde":
        return None, None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), key=_profile_order)
    for f in reversed(files):
        try:
            lab = json.load(open(f)).get("bench_labels", {}).get(kernel)
        except (OSError, ValueError):
            continue
        if not lab:
            continue
        traffic = lab.get("hbm_bytes_per_launch")
        valu = None
        if lab.get("valu_wave_instr_per_launch"):
            rate = lab["valu_wave_instr_per_launch"] / (avg_ms * 1e-3)
            valu = {"kernel": kernel, "wave_instr_per_launch": lab["valu_wave_instr_per_launch"],
                    "achieved": round(rate / 1e9, 1), "peak": VALU_PEAK_WAVE_INSTR_S / 1e9,
                    "unit": "G wave-instr/s", "frac": round(rate / VALU_PEAK_WAVE_INSTR_S, 4),
                    "source": os.path.basename(f)}
        return traffic, valu
    return None, None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import zkgpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    zkgpu.init(local)
    stream = torch.cuda.current_stream()
    zkgpu.set_stream(stream)

    n = 1 << args.log_n
    ne = n << args.blowup_bits
    C = args.ncols
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + rank)
    # canonical Goldilocks values: uniform in [0, 2^63) < p
    gs = None
    if args.workload == "commit":
        from zkgpu.sharded import ShardedCommit, col_range
        lo, hi = col_range(C, world, rank)
        trace = torch.randint(0, 2**63 - 1, (max(hi - lo, 1), n), dtype=torch.int64, device=dev, generator=g)
        sc = ShardedCommit(args.log_n, args.blowup_bits, C, device=dev)

        def step():
            sc.commit(trace)
    elif args.workload == "stark":
        from zkgpu.stark import GpuStark
        inst = stark_instance(args.log_n, args.blowup_bits, C, args.queries)
        gs = GpuStark(inst)  # setup: constants, constant LDE + tree (untimed, loaded from files in the reference)
        gs.witness()         # executor stand-in: committed trace cm1 in HBM (untimed)

        def step():
            gs.prove_raw()
    elif args.workload == "stark-sharded":
        # ONE proof of one trace for the whole job, extended domain row-sharded over the ranks
        from zkgpu.sharded_stark import ShardedStark
        inst = stark_instance(args.log_n, args.blowup_bits, C, args.queries)
        ss = ShardedStark(inst, device=dev)  # setup: constants + sharded constant tree (untimed)
        ss.witness()                         # executor stand-in (untimed)

        def step():
            ss.prove()
    elif args.workload == "lde":
        trace = torch.randint(0, 2**63 - 1, (C, n), dtype=torch.int64, device=dev, generator=g)
        out = torch.empty((C, ne), dtype=torch.int64, device=dev)

        def step():
            zkgpu.extend_pol_dev(out, ne, trace, n, ne, n, C)
    else:
        rows = n
        src = torch.randint(0, 2**63 - 1, (C, rows), dtype=torch.int64, device=dev, generator=g)
        nodes = torch.empty(zkgpu.merkle_num_elements(rows), dtype=torch.int64, device=dev)

        def step():
            zkgpu.merkletree_dev(nodes, src, rows, C, rows)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    zkgpu.prof_reset()
    zkgpu.prof_enable(True)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    zkgpu.prof_enable(False)

    # per-kernel live timings (HIP events on the launch stream)
    kernels = {}
    for k in zkgpu.prof_kernels():
        launches, ms, by = zkgpu.prof_query(k)
        kernels[k] = (launches, ms, by)
    dom = max(kernels, key=lambda k: kernels[k][1])
    launches, ms, by = kernels[dom]
    avg_ms = ms / launches
    achieved = (by / launches) / (avg_ms * 1e-3) / 1e9
    traffic, valu = pmc_for(dom, args, avg_ms)

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    if rank == 0:
        if args.workload == "commit":
            total_elems = ne * C * args.steps  # one trace for the whole job
            unit, metric_unit = "Gelem/s", "LDE elements committed (LDE + Merkle)"
            alg_step = (8 * (n + ne) * C + 8 * ne * C + 32 * ne + 96 * ne) // world
        elif args.workload == "stark":
            total_elems = world * args.steps
            unit, metric_unit = "s/proof", "proofs"
            alg_step = 8 * (n + ne) * (C + 48 + 6)
        elif args.workload == "stark-sharded":
            total_elems = args.steps  # one proof per step for the whole job
            unit, metric_unit = "s/proof", "proofs"
            alg_step = 8 * (n + ne) * (C + 48 + 6) // world
        elif args.workload == "lde":
            total_elems = ne * C * world * args.steps
            unit, metric_unit = "Gelem/s", "LDE output elements"
            alg_step = 8 * (n + ne) * C  # per step per GPU
        else:
            total_elems = n * C * world * args.steps
            unit, metric_unit = "Gelem/s", "Merkle leaf elements hashed"
            alg_step = 8 * n * C + 32 * n + 96 * (n - 1)
        value = total_elems / elapsed / 1e9
        if args.workload in ("stark", "stark-sharded"):
            value = elapsed / total_elems  # seconds per proof, whole job
        cpu = None
        if world == 1 and not args.no_cpu and args.workload == "commit":
            cpu = cpu_baseline_commit(args.log_n, args.blowup_bits, C, args.cpu_sample_bits)
        if world == 1 and not args.no_cpu and args.workload == "stark":
            cpu = cpu_baseline_stark(args.cpu_sample_bits, args.log_n, args.blowup_bits, C, args.queries)
        if world == 1 and not args.no_cpu and args.workload == "lde":
            cpu = cpu_baseline(args.log_n, args.blowup_bits, args.cpu_sample_cols)
        if world == 1 and not args.no_cpu and args.workload == "merkle":
            cpu = cpu_baseline_merkle(args.log_n, C)
        if args.workload == "lde":
            workload = ("LDE 2^%d -> 2^%d rows x %d cols per GPU (extendPol, starks.cpp:53), column-major in HBM"
                        % (args.log_n, args.log_n + args.blowup_bits, C))
        elif args.workload == "commit":
            workload = ("column-sharded commit of one 2^%d-row x %d-col trace over %d rank(s): LDE 2^%d -> 2^%d, "
                        "all-to-all column->row blocks, per-rank Merkle subtree, sub-root gather + top levels "
                        "(starks.cpp:53-57)" % (args.log_n, C, world, args.log_n, args.log_n + args.blowup_bits))
        elif args.workload == "merkle":
            workload = ("Poseidon-GL Merkle tree over 2^%d rows x %d cols per GPU (merkelize, merkleTreeGL.cpp:37-44)"
                        % (args.log_n, C))
        else:
            workload = ("full STARK proof (genProof stages 1-5 + FRI + queries, starks.cpp:9-404), synthetic "
                        "config-4 instance: 2^%d trace, blowup 2^%d, cm1/cm2/cm3/cm4 = %d/%d/%d/%d, %d constants, "
                        "2 plookups (dim 3 + dim 1), FRI steps %s, %d queries; one independent proof per GPU"
                        % (args.log_n, args.blowup_bits, inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4,
                           inst.n_const, inst.fri_steps, args.queries))
            if args.workload == "stark-sharded":
                workload = workload.replace("one independent proof per GPU",
                                            "ONE proof for the whole job, row-sharded over %d rank(s)" % world)
        res = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": unit,
            "value_meaning": ((metric_unit + " per second, all GPUs") if not args.workload.startswith("stark")
                              else "wall seconds per proof, whole job"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": not args.workload.startswith("stark"),
            "scaling": "strong" if args.workload in ("commit", "stark-sharded") else "weak",
            "vs_baseline": None,
            "dtype": "u64 (Goldilocks)" if not args.workload.startswith("stark") else "u64 (Goldilocks) + F_p^3",
            "data": "synthetic (uniform canonical Goldilocks, torch generator seed 0x5EED+rank)",
            "config": {
                "workload": workload,
                "log_n": args.log_n, "blowup_bits": args.blowup_bits, "ncols_per_gpu": C,
                "parallelism": {"stark": "replicas x%d (one independent proof per GPU)" % world,
                                "stark-sharded": ("one proof, extended domain row-sharded x%d: RCCL all-to-all "
                                                  "column->row blocks per commit, halo + q/f all-gathers" % world),
                                "commit": "column-sharded x%d, RCCL all-to-all column->row blocks" % world}.get(
                    args.workload, "column-sharded x%d (no data-path collective)" % world),
            },
            "valu": valu,
            "roofline": {
                "kernel": dom,
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "avg_launch_ms": round(avg_ms, 4),
                "alg_bytes_per_launch": by / launches,
                "step_frac": round(alg_step / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
            },
            "kernels": {k: {"launches": v[0], "avg_ms": round(v[1] / v[0], 4),
                            "GB/s": round(v[2] / v[0] / (v[1] / v[0] * 1e-3) / 1e9, 1)} for k, v in kernels.items()},
            "cpu_baseline": cpu,
        }
        if gs is not None:
            res["stages_ms"] = {k: round(v, 3) for k, v in gs.timers().items()}
        if args.workload == "stark-sharded":
            res["stages_ms"] = {k: round(v, 3) for k, v in ss.timers.items()}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
