#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X STARK hot path.

BASELINE.json metric: "batch-proof STARK sec (2^23 trace) + Goldilocks NTT
Gelem/s at 1/2/4/8 GPU".

Default workload (configs[3], the north star): one full STARK proof
(Starks::genProof stages 1-5 + FRI + queries, starks.cpp:9-404) of the
synthetic config-4 instance -- 2^23-row trace, blowup 2, cm1/cm2/cm3/cm4 =
100/26/27/6 columns, 30 constants, two plookups, a post-Z step3, FRI steps
[24, 20, 16, 12, 8, 5], 128 queries -- with the committed trace resident in
HBM (the executor stand-in runs before the timed region; the constant LDE and
tree are setup, as the reference loads them from files).  One step = one
proof.  value = wall seconds per proof (whole job; lower is better).
Multi-GPU (N > 1): the headline is ONE config-4 proof over all N ranks
(configs[4], strong scaling; sharded_one_proof.config4, measured by child
processes over RCCL); the replica throughput (one independent proof per GPU)
is reported beside it as `replicas`, and is the value only if the one-proof
run failed (the line says so).

The same line carries the Goldilocks NTT number of the metric, measured in the
same process after the proofs: the LDE of configs[1] (2^23 -> 2^24 x 100
columns, extendPol, starks.cpp:53), as `lde` (Gelem/s) -- and the LDE is the
kernel chain `roofline` describes (algorithmic bytes per LDE =
24 N C; achieved = that / the device time of the LDE's NTT passes, HIP events
on the launch stream).  Poseidon Merkle hashing, the largest share of the
proof, is integer-VALU bound; `valu` prices its kernel against the measured
issue peak (tools/instbench.hip, profiles/*_instbench.json).

cpu_baseline: the oracle's STARK prover (C/OpenMP kernels, kind "port") on a
bounded sample of the same instance shape (2^--cpu-sample-bits rows), rank 0
at N=1; `full_size` quotes the committed measurement of the oracle at 2^23
(`bench.py --cpu-full`, profiles/*_cpu_full_stark.json) when one exists.

  python bench.py [--gpus N] [--steps K] [--warmup W]
                  [--workload stark|lde|merkle|stark-sharded|step42ns] [--zkevm-shaped] [--no-cpu] [--no-lde]
"""
import argparse
import glob
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zkevm-prover_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CLOCK_HZ = 2.4e9       # MI355X_MICROARCH.md: max clock 2400 MHz
N_SIMDS = 256 * 4      # 256 CUs x 4 SIMDs
METRIC = "batch-proof STARK sec (2^23 trace) + Goldilocks NTT Gelem/s at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ncols", type=int, default=100)
    ap.add_argument("--log-n", type=int, default=23)
    ap.add_argument("--blowup-bits", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-lde", action="store_true", help="skip the secondary LDE measurement (stark workload)")
    ap.add_argument("--no-handoff", action="store_true",
                    help="skip the host->device trace hand-off timing (stark workload, N=1)")
    ap.add_argument("--lde-steps", type=int, default=10)
    ap.add_argument("--workload", choices=["stark", "lde", "merkle", "stark-sharded", "step42ns"],
                    default="stark",
                    help="stark = configs[3] (headline: full synthetic STARK proof, 2^23 trace); lde = configs[1] "
                         "(2^23 -> 2^24 x 100 LDE); merkle = configs[2] (2^23 x 100 Poseidon tree); stark-sharded = "
                         "configs[4] (one proof over all ranks, strong scaling); step42ns = the quotient program of "
                         "the reference's zkEVM shape on the 2^(log_n+1) extended domain")
    ap.add_argument("--queries", type=int, default=128)
    ap.add_argument("--no-sharded", action="store_true",
                    help="stark workload: skip the one-proof-over-all-ranks measurement (configs[4])")
    ap.add_argument("--sharded-timeout", type=int, default=150,
                    help="seconds each sharded child run may take before it is killed and reported as failed")
    ap.add_argument("--fork9", action="store_true",
                    help="stark / stark-sharded: the fork-9 widths (751/168/408/6 committed, 234 constants, 389 "
                         "tmpExp; SyntheticStark.fork9) instead of config-4's")
    ap.add_argument("--zkevm-shaped", action="store_true",
                    help="stark / stark-sharded: the fork-9 widths with the five zkEVM-shaped expression programs "
                         "(zkgpu/zkevm_shaped.py: step2prev / step3prev / step3 / step42ns / step52ns in the stage "
                         "slots, 1,973 evaluations)")
    ap.add_argument("--s42-scale", type=float, default=1.0,
                    help="step42ns workload: fraction of the reference step42ns opcode counts")
    ap.add_argument("--s42-jit", action="store_true", help="step42ns workload: the compiled kernel (else interpreter)")
    ap.add_argument("--no-s42", action="store_true",
                    help="stark workload: skip the zkEVM-shaped quotient block (quotient_zkevm_shaped)")
    ap.add_argument("--s42-steps", type=int, default=3)
    ap.add_argument("--no-cpu-zkevm", action="store_true",
                    help="stark workload: skip the oracle's zkEVM-shaped sample (cpu_baseline.zkevm_shaped, 2^16 rows, ~20 s)")
    ap.add_argument("--cpu-sample-bits", type=int, default=int(os.environ.get("ZKGPU_CPU_SAMPLE_BITS", "18")))
    ap.add_argument("--cpu-sample-cols", type=int, default=int(os.environ.get("ZKGPU_CPU_SAMPLE_COLS", "4")))
    ap.add_argument("--comm", choices=["rccl", "shm"], default="rccl",
                    help="stark-sharded: the exchange -- RCCL over xGMI, or host shared memory (zkgpu_comm_host, the "
                         "fallback the default bench retries with when the RCCL run fails)")
    ap.add_argument("--rank-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-full", action="store_true",
                    help="only time the oracle STARK prover at the full size (minutes of CPU); prints one JSON line "
                         "for profiles/*_cpu_full_stark.json")
    return ap.parse_args()


# ---------------------------------------------------------------- instances
def stark_instance(log_n, blow, ncols, n_queries, fork9=False):
    """cm1 = ncols, cm2 = 26, cm3 = 27, cm4 = 6, 30
    constants, qDeg 2, FRI steps [nBitsExt, -4, ..., 5], n_queries queries
    (synthetic AIR, zkgpu/synthetic.py); fork9: the zkEVM's widths;
    fork9 = "zkevm": those widths with the five zkEVM-shaped expression
    programs (zkgpu/zkevm_shaped.py)."""
    from zkgpu.synthetic import SyntheticStark
    nbe = log_n + blow
    steps = [nbe]
    while steps[-1] - 4 >= 5:
        steps.append(steps[-1] - 4)
    if steps[-1] > 5:
        steps.append(5)
    if fork9 == "zkevm":
        from zkgpu.zkevm_shaped import ZkevmShapedStark
        return ZkevmShapedStark.create(n_bits=log_n, n_queries=n_queries, fri_steps=steps)
    if fork9:
        return SyntheticStark.fork9(n_bits=log_n, n_queries=n_queries, fri_steps=steps)
    # cm1 = 3t constrained triples + free columns + 3 lookup columns (A, B, C);
    # cm2 = 6 h groups (18) + plookup h1/h2 (3+3+1+1) = 26; cm3 = 18 + 2 plookup
    # Z + the step3 column W = 27; constants = 26 K + L_first + 3 tables = 30
    t = (ncols - 3) // 3
    return SyntheticStark(n_bits=log_n, blowup_bits=blow, t=t, n_free=ncols - 3 - 3 * t, m=6, n_k=26,
                          n_queries=n_queries, fri_steps=steps, n_lookups=2)


def _kind(args):
    """stark_instance's fork9 argument from the command line"""
    return "zkevm" if getattr(args, "zkevm_shaped", False) else args.fork9


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)


# ---------------------------------------------------------------- CPU baselines (oracle = checker only)
# what the CPU baseline is: the checker, not the reference's CPU path
PORT_NOTE = ("oracle port (scalar C + OpenMP, the textbook dense 12x12 MDS in every Poseidon round), not the "
             "reference's AVX2 Goldilocks path (absent submodule, unbuildable here): a GPU/CPU ratio against it "
             "overstates the lead over the reference")


REF_NOTE = ("the reference's default CPU path restated (cpuref/cpuref.cpp: AVX2 Goldilocks arithmetic, Poseidon "
            "with the sparse partial rounds over 4 states per vector, merkletree_avx's OpenMP over rows, the blocked "
            "row-major NTT of build_const_tree.cpp:216-533 vectorised over columns, the Steps programs 4 rows per "
            "AVX2 step as the reference's parser); the proof orchestration, evmap, H1H2, Z and FRI stay the oracle's "
            "(oracle/stark_prover.py), bit-identical kernels (tests/test_cpuref.py); the goldilocks submodule itself "
            "is absent, so this is a restatement, not the reference's binary")


def _cpu_prove(inst, fast):
    """wall seconds of one oracle-orchestrated proof; fast: cpuref's kernels"""
    from oracle import oracle as oc
    from oracle.stark_prover import OracleStark
    sys.path.insert(0, os.path.join(ROOT, "cpuref"))
    import cpuref
    threads = _threads()
    oc.lib().oc_set_num_threads(threads)
    cpuref.lib().cr_set_num_threads(threads)
    import contextlib
    with (cpuref.as_oracle_kernels(oc) if fast else contextlib.nullcontext()):
        o = OracleStark(inst)
        o.witness()
        t0 = time.perf_counter()
        o.prove()
        return time.perf_counter() - t0


def cpu_baseline_stark(sample_bits, blow, ncols, n_queries):
    """The reference's CPU path restated (cpuref) on the same instance shape
    at 2^sample_bits rows; the oracle port's time beside it."""
    threads = _threads()
    inst = stark_instance(sample_bits, blow, ncols, n_queries)
    dt = _cpu_prove(inst, True)
    dp = _cpu_prove(inst, False)
    return {"value": round(dt, 3), "unit": "s/proof", "cores": threads, "kind": "restated-reference-AVX2",
            "what": REF_NOTE,
            "sample": "genProof of the config-4 instance shape at 2^%d rows (%d cm1 cols, %d queries), %.1f s, %d "
                      "threads (%s)" % (sample_bits, ncols, n_queries, dt, threads, _cpu_model()),
            "port": {"value": round(dp, 3), "unit": "s/proof", "kind": "port", "what": PORT_NOTE,
                     "sample": "the same proof through the oracle's own kernels (scalar C + OpenMP), %.1f s" % dp}}


def cpu_baseline_zkevm(sample_bits, n_queries):
    """The reference's CPU path restated (cpuref) on the zkEVM-shaped instance
    (fork-9 widths + the five zkEVM-shaped programs, zkgpu/zkevm_shaped.py) at
    2^sample_bits rows: the CPU path of the same proof the GPU's
    sharded_one_proof.fork9_zkevm_shaped line times at 2^23."""
    threads = _threads()
    inst = stark_instance(sample_bits, 1, 100, n_queries, "zkevm")
    dt = _cpu_prove(inst, True)
    return {"value": round(dt, 3), "unit": "s/proof", "cores": threads, "kind": "restated-reference-AVX2",
            "what": REF_NOTE, "rows": 1 << sample_bits,
            "sample": "oracle genProof of the zkEVM-shaped instance (751/168/408/6 committed, 234 constants, the five "
                      "zkEVM-shaped programs, 1,973 evaluations) at 2^%d rows, %d queries, %.1f s, %d threads (%s)"
                      % (sample_bits, n_queries, dt, threads, _cpu_model())}


def cpu_full_size_record():
    """The committed full-size oracle measurement (bench.py --cpu-full), newest."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_cpu_full_stark.json")), key=_profile_order)
    for f in reversed(files):
        try:
            d = json.load(open(f))
            d["source"] = "profiles/" + os.path.basename(f)
            return d
        except (OSError, ValueError):
            continue
    return None


def _cpuref():
    sys.path.insert(0, os.path.join(ROOT, "cpuref"))
    import cpuref
    cpuref.lib().cr_set_num_threads(_threads())
    return cpuref


def cpu_baseline_lde(log_n, blow, ncols_sample):
    """extendPol on the host cores, the reference's path restated (cpuref), on
    a bounded sample: 2^log_n -> 2^(log_n+blow) x ncols_sample."""
    import numpy as np
    cr = _cpuref()
    threads = _threads()
    rng = np.random.default_rng(0x5EED)
    x = rng.integers(0, 2**63, size=(1 << log_n, ncols_sample), dtype=np.uint64)
    t0 = time.perf_counter()
    cr.extend_pol(x, 1 << (log_n + blow))
    dt = time.perf_counter() - t0
    out_elems = (1 << (log_n + blow)) * ncols_sample
    return {"value": out_elems / dt / 1e9, "unit": "Gelem/s", "cores": threads, "kind": "restated-reference-AVX2",
            "what": REF_NOTE,
            "sample": "extendPol 2^%d->2^%d x %d cols, %.1f s, %d threads (%s)"
                      % (log_n, log_n + blow, ncols_sample, dt, threads, _cpu_model())}


def cpu_baseline_merkle(log_n, ncols):
    """merkelize on the host cores, the reference's merkletree_avx restated
    (cpuref), on 2^min(log_n, 18) rows"""
    import numpy as np
    cr = _cpuref()
    threads = _threads()
    rows = 1 << min(log_n, 18)
    rng = np.random.default_rng(0x5EED)
    x = rng.integers(0, 2**63, size=(rows, ncols), dtype=np.uint64)
    t0 = time.perf_counter()
    cr.merkletree(x)
    dt = time.perf_counter() - t0
    return {"value": rows * ncols / dt / 1e9, "unit": "Gelem/s", "cores": threads, "kind": "restated-reference-AVX2",
            "what": REF_NOTE,
            "sample": "merkletree 2^%d rows x %d cols, %.1f s, %d threads (%s)"
                      % (min(log_n, 18), ncols, dt, threads, _cpu_model())}


# ---------------------------------------------------------------- committed profiles
def _profile_order(path):
    """Natural order of profiles/rNN_vM_* names (r02_v10 after r02_v9); the
    newest summary wins.  File mtimes are not used: a fresh checkout or a
    gpurun snapshot gives every file the same one."""
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]


def _newest(pattern, load=True):
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=_profile_order)
    if not load:
        return (files[-1], None) if files else (None, None)
    for f in reversed(files):
        try:
            return f, json.load(open(f))
        except (OSError, ValueError):
            continue
    return None, None


def _stamped(pattern, family):
    """(path, doc, note) of the newest profile matching pattern whose source
    stamp (zkgpu/stamp.py) matches the current sources of `family`; when none
    does: (newest path, None, why) -- the counters describe other kernels and
    are not used."""
    from zkgpu.stamp import check
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=_profile_order)
    stale = None
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        ok, why = check(d, family)
        if ok:
            return f, d, why
        if stale is None:
            stale = (f, None, "stale: %s (%s)" % (why, os.path.basename(f)))
    return stale or (None, None, "no committed %s profile" % pattern)


def valu_peak(kernel, family):
    """Issue peak of `kernel` in wave64 VALU instructions / s: the measured
    per-instruction issue cost at 8 waves per SIMD (profiles/*_instbench.json,
    tools/instbench.hip) weighted by the kernel's static VALU instruction mix
    (profiles/*_valu_mix.json, tools/valu_mix.py over the shipped code object,
    stamped).  Returns (peak, note) or (None, reason)."""
    fi, ib = _newest("*_instbench.json")
    fm, mix, why = _stamped("*_valu_mix.json", family)
    if not ib:
        return None, "no committed instbench profile"
    cost = {}
    for r in ib["rows"]:
        if r["waves_per_simd"] == 8:
            cost[r["instr"]] = r.get("cycles", r.get("cycles_at_2p4GHz"))
    base = cost.get("v_add_u32")
    km = (mix or {}).get("kernels", {}).get(kernel)
    if not km:
        return N_SIMDS * CLOCK_HZ / base, "v_add_u32 issue cost %.2f clk (8 waves/SIMD); no current mix for %s (%s)" % (
            base, kernel, why)
    tot, cyc = 0, 0.0
    for ins, n in km["histogram"].items():
        c = cost.get(ins, base)  # instructions not measured separately: the v_add_u32 rate
        tot += n
        cyc += n * c
    avg = cyc / tot
    return N_SIMDS * CLOCK_HZ / avg, ("mix-weighted issue cost %.3f clk per wave64 VALU instruction (8 waves/SIMD, "
                                      "%s x %s)" % (avg, os.path.basename(fi), os.path.basename(fm)))


def lde_traffic_per_lde(labels_launches):
    """PMC HBM bytes of one LDE: sum over its pass kernels of the per-launch
    traffic in the newest profiles/*_lde_pmc.json (separate FETCH_SIZE /
    WRITE_SIZE passes of `bench.py --workload lde`, gfx950 corrections) --
    only when its stamp matches the current NTT sources.  Returns (bytes,
    source, note)."""
    f, d, why = _stamped("*_lde_pmc.json", "lde")
    if not d:
        return None, None, why
    labs = d.get("bench_labels", {})
    tot = 0.0
    for lab, n in labels_launches.items():
        if lab not in labs or "hbm_bytes_per_launch" not in labs[lab]:
            return None, None, "the profile has no %s" % lab
        tot += labs[lab]["hbm_bytes_per_launch"] * n
    return tot, os.path.basename(f), why


def kernel_counters(kernel, family, launches_per_proof):
    """VALU wave-instructions and HBM bytes of one proof's launches of
    `kernel` in the newest stamped profiles/*_stark_pmc.json (the last
    launches_per_proof launches of its one-proof run: the earlier ones are
    setup) and the kernel's clock there.  Returns (dict, note) or (None, why)."""
    f, d, why = _stamped("*_stark_pmc.json", family)
    if not d:
        return None, why
    k = d.get("kernels", {}).get(kernel)
    if not k or "launch_valu" not in k:
        return None, "the profile has no per-launch record of %s" % kernel
    lv, lm = k["launch_valu"][-launches_per_proof:], k["launch_ms"][-launches_per_proof:]
    return {"valu_per_proof": sum(lv), "pmc_ms_per_proof": sum(lm), "launches": len(lv),
            "hbm_bytes_per_launch": k.get("hbm_bytes_per_launch"),
            "clock_GHz": k.get("clock_GHz") if k.get("clock_valid") else None,
            "source": os.path.basename(f)}, why


def stark_valu(kernel, ms_per_proof, launches_per_proof, family="poseidon"):
    """VALU issue rate of `kernel` in this run: its stamped per-proof
    SQ_INSTS_VALU over its device time per proof here, against the
    mix-weighted issue peak; the clock the kernel runs at (GRBM busy cycles /
    kernel time, kept only when <= the 2.4 GHz maximum)."""
    kc, why = kernel_counters(kernel, family, launches_per_proof)
    if kc is None:
        return {"kernel": kernel, "stale": True, "note": why}
    peak, note = valu_peak(kernel, family)
    if peak is None:
        return None
    rate = kc["valu_per_proof"] / (ms_per_proof * 1e-3)
    frac = rate / peak
    if frac > 1.0:
        raise SystemExit("valu.frac %.3f > 1 for %s: the peak model (%s) is wrong" % (frac, kernel, note))
    res = {"kernel": kernel, "wave_instr_per_proof": kc["valu_per_proof"], "launches_per_proof": launches_per_proof,
           "ms_per_proof": round(ms_per_proof, 3), "achieved": round(rate / 1e9, 1), "peak": round(peak / 1e9, 1),
           "unit": "G wave-instr/s", "frac": round(frac, 4),
           "peak_model": note + " at the nominal %.1f GHz" % (CLOCK_HZ / 1e9), "source": kc["source"],
           "stamp": why}
    ghz = kc["clock_GHz"]
    if ghz and ghz <= CLOCK_HZ / 1e9:
        res["clock_GHz"] = ghz
        res["peak_at_clock"] = round(peak * ghz * 1e9 / CLOCK_HZ / 1e9, 1)
        res["frac_at_clock"] = round(frac * CLOCK_HZ / (ghz * 1e9), 4)
    return res


# ---------------------------------------------------------------- timing helpers
def timed(step, steps, warmup, world, dist, torch, prepare=None):
    """K steps bracketed by a barrier + synchronize on both sides.  With
    `prepare` (a step that consumes its input: the lean-plan prover extends
    the trace in place), each step gets its own bracket and prepare() runs
    between them, outside the timing; elapsed = the sum of the brackets."""
    for _ in range(warmup):
        if prepare:
            prepare()
        step()
    torch.cuda.synchronize()
    import zkgpu
    zkgpu.prof_reset()
    if prepare is None:
        zkgpu.prof_enable(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    else:
        elapsed = 0.0
        for _ in range(steps):
            prepare()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            zkgpu.prof_enable(True)
            t0 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            elapsed += time.perf_counter() - t0
            zkgpu.prof_enable(False)
    zkgpu.prof_enable(False)
    kernels = {}
    for k in zkgpu.prof_kernels():
        kernels[k] = zkgpu.prof_query(k)  # (launches, ms, bytes)
    return elapsed, kernels


def max_over_ranks(x, world, dist, torch, dev):
    t = torch.tensor([x], dtype=torch.float64, device=_coll_dev(dist) if world > 1 else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def kernel_table(kernels):
    return {k: {"launches": v[0], "avg_ms": round(v[1] / v[0], 4),
                "GB/s": round(v[2] / v[0] / (v[1] / v[0] * 1e-3) / 1e9, 1)} for k, v in kernels.items() if v[0]}


def lde_measure(args, dev, torch, world, dist):
    """configs[1]: LDE 2^log_n -> 2^(log_n+blow) x ncols, column-major in HBM.
    Returns (lde dict, roofline dict)."""
    import zkgpu
    n = 1 << args.log_n
    ne = n << args.blowup_bits
    C = args.ncols
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + int(os.environ.get("RANK", "0")))
    trace = torch.randint(0, 2**63 - 1, (C, n), dtype=torch.int64, device=dev, generator=g)
    out = torch.empty((C, ne), dtype=torch.int64, device=dev)
    steps = args.steps if args.workload == "lde" else args.lde_steps

    def step():
        zkgpu.extend_pol_dev(out, ne, trace, n, ne, n, C)

    elapsed, kernels = timed(step, steps, 2 if args.workload != "lde" else args.warmup, world, dist, torch)
    elapsed = max_over_ranks(elapsed, world, dist, torch, dev)
    passes = {k: v for k, v in kernels.items() if k.startswith(("k_ntt_pass", "k_lde_")) or k == "k_ntt_small"}
    dev_ms = sum(v[1] for v in passes.values()) / steps
    alg = 24.0 * n * C if args.blowup_bits == 1 else 8.0 * (n + ne) * C
    achieved = alg / (dev_ms * 1e-3) / 1e9
    launches = {k: v[0] / steps for k, v in passes.items()}
    traffic, src, tnote = None, None, "counters exist for configs[1] only (2^23 -> 2^24 x 100)"
    if args.log_n == 23 and C == 100 and args.blowup_bits == 1:
        traffic, src, tnote = lde_traffic_per_lde(launches)
    roof = {"kernel": "extendPol = NTT pass chain (%s per LDE)"
                      % ", ".join("%g x %s" % (launches[k], k) for k in sorted(launches)),
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic, "traffic_ratio": round(traffic / alg, 2) if traffic else None,
            "traffic_source": src, "traffic_stamp": tnote, "alg_bytes_per_launch": alg,
            "alg_bytes_note": "SURVEY.md 8(d): LDE N -> 2N x C reads 8NC, writes 16NC = 24NC bytes; 'launch' = "
                              "one LDE (its NTT pass kernels), device time from HIP events on the launch stream",
            "avg_launch_ms": round(dev_ms, 4)}
    lde = {"value": round(ne * C * world * steps / elapsed / 1e9, 3), "unit": "Gelem/s",
           "meaning": "LDE output elements per second, all GPUs (configs[1]: 2^%d -> 2^%d x %d cols per GPU)"
                      % (args.log_n, args.log_n + args.blowup_bits, C),
           "ms_per_lde": round(elapsed / steps * 1e3, 4), "device_ms_per_lde": round(dev_ms, 4), "steps": steps,
           "kernels": kernel_table(passes)}
    del trace, out
    torch.cuda.empty_cache()
    return lde, roof


def step42ns_setup(args, dev, torch, g):
    """The step42ns-shaped program (zkgpu/synthetic_bytecode.py, seed 1) on
    the 2^(log_n+1)-row extended domain: cm1/cm2/cm3/cm4/const 2ns sections of
    the fork-9 widths in HBM (about 12.5 KB per row), q_2ns written."""
    import numpy as np
    import zkgpu
    import zkgpu.parser as zp
    import zkgpu.synthetic_bytecode as sb
    shape = sb.load_shape()
    ops, a = sb.generate("step42ns", seed=1, scale=args.s42_scale)
    secs = sb.sections(shape)
    prog = zp.convert(zp.STEP42NS, ops, a, secs, shape["n_bits"], shape["n_bits_ext"])
    log_dom = args.log_n + 1
    NE = 1 << log_dom
    LD = NE + int(os.environ.get("ZKGPU_S42_PAD", "0"))  # column stride (A/B of padded sections)
    dsecs = {}
    cols = 0
    for sec, _, w in secs:
        if sec >= 5:
            dsecs[sec] = (torch.randint(0, 2**63 - 1, (w, LD), dtype=torch.int64, device=dev, generator=g), LD, w)
            cols += w
    dsecs[9] = (torch.randint(0, 2**63 - 1, (shape["n_const"], LD), dtype=torch.int64, device=dev, generator=g), LD,
                shape["n_const"])
    cols += shape["n_const"]
    q = torch.zeros((3, NE), dtype=torch.int64, device=dev)
    dsecs[10] = (q, NE, 3)
    rng = np.random.default_rng(42)
    P = 0xFFFFFFFF00000001
    chal = rng.integers(0, P, (8, 3), dtype=np.uint64)
    pub = rng.integers(0, P, 48, dtype=np.uint64)
    evals = rng.integers(0, P, (4, 3), dtype=np.uint64)

    def step():
        zkgpu.zxp_eval_dev(prog, dsecs, log_dom, chal, pub, evals, extend_bits=1, x_start=7)

    # default: the interpreter.  --s42-jit times the compiled kernel: scale
    # 0.25 is cached by build(), the full-size kernel (~10 min of hiprtc) by
    # tools/jit_prebuild.py --full
    os.environ["ZKGPU_ZXP_JIT"] = "2" if args.s42_jit else "0"
    # the distinct element reads per row -- every (section,
    # column, row shift) the program reads once -- plus the 3 q columns written
    ins, opn = prog.arrays()
    reads = set()
    for kind, a_, b_, c_ in opn.tolist():
        if kind in (2, 3):  # ZXP_COL / ZXP_COL3
            for j in range(3 if kind == 3 else 1):
                reads.add((a_, b_ + j, c_))
    return step, {"rows": NE, "log_dom": log_dom, "n_ops": int(len(ops)), "cols_read": len(reads),
                  "cols_alloc": cols, "alg_bytes": 8.0 * NE * (len(reads) + 3), "tensors": dsecs}


def step42ns_roofline(s42, kernels, steps):
    """HBM roofline of the compiled quotient kernel: every section column
    read once + q written (8 B each per row) / its device time per launch."""
    ks = {k: v for k, v in kernels.items() if k.startswith("k_zxp_jit") or k == "k_zxp_eval"}  # compiled / interpreter
    if not ks:
        return None
    dev_ms = sum(v[1] for v in ks.values()) / steps
    achieved = s42["alg_bytes"] / (dev_ms * 1e-3) / 1e9
    return {"kernel": ", ".join(sorted(ks)), "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "alg_bytes_per_launch": s42["alg_bytes"],
            "alg_bytes_note": "SURVEY.md 8(d): 8 B x rows x (%d distinct (section, column, row shift) reads + 3 q "
                              "columns written)" % s42["cols_read"],
            "avg_launch_ms": round(dev_ms, 4)}


def leaves_line(inst, args, v):
    """The dominant kernel of the proof, k_leaves_cols (the Merkle leaf hash
    of each commit, linear_hash per row, merkleTreeGL.cpp:37-44), on both of
    its bounds: HBM (8 B x rows x cols + 32 B digest per row)
    and permutations per second against the isolated permutation benchmark
    (tools/poseidon_bench.hip, profiles/*_poseidon_bench.txt)."""
    ne = 1 << (args.log_n + args.blowup_bits)
    widths = [inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4]
    launches, ms = v[0] / args.steps, v[1] / args.steps  # per proof
    alg = sum(8.0 * ne * w + 32.0 * ne for w in widths)
    perms = sum(ne * ((w + 7) // 8) for w in widths)
    res = {"kernel": "k_leaves_cols", "launches_per_proof": launches, "ms_per_proof": round(ms, 3),
           "avg_launch_ms": round(ms / launches, 4), "widths": widths, "rows": ne,
           "alg_bytes_per_proof": alg, "achieved_GBs": round(alg / (ms * 1e-3) / 1e9, 1),
           "hbm_frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "perms_per_proof": perms, "Gperm_s": round(perms / (ms * 1e-3) / 1e9, 3),
           "bound": "VALU (~20 K VALU per 64 B absorbed; the valu block prices it against the issue peak)"}
    f, d, why = _stamped("*_poseidon_bench.json", "poseidon")
    if d and d.get("fast_Gperm_s"):
        res["isolated_Gperm_s"] = d["fast_Gperm_s"]
        res["ratio_to_isolated"] = round(res["Gperm_s"] / d["fast_Gperm_s"], 3)
        res["isolated_source"] = "%s (the shipped permutation, one state per thread, %s GHz under load; %s)" % (
            os.path.basename(f), d.get("clock_GHz"), why)
    else:
        res["isolated_note"] = why
    return res


def dominant_roofline(inst, args, v, valu):
    """k_leaves_cols, the proof's dominant kernel, on both of its bounds from
    this run's timing: HBM (SURVEY.md 8(d) leaves bytes: 8 B x rows x cols +
    32 B digest per row, per proof) and VALU issue (the stamped per-proof
    SQ_INSTS_VALU of the same build, the valu block)."""
    ne = 1 << (args.log_n + args.blowup_bits)
    widths = [inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4]
    ms = v[1] / args.steps
    alg = sum(8.0 * ne * w + 32.0 * ne for w in widths)
    hbm = alg / (ms * 1e-3) / 1e9
    res = {"kernel": "k_leaves_cols", "ms_per_proof": round(ms, 3), "bound": "valu",
           "hbm": {"achieved": round(hbm, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(hbm / HBM_PEAK_GBS, 4),
                   "alg_bytes_per_proof": alg}}
    if valu and not valu.get("stale"):
        res["valu"] = {k: valu[k] for k in ("achieved", "peak", "unit", "frac", "frac_at_clock", "clock_GHz", "source")
                       if k in valu}
    else:
        res["valu"] = {"stale": True, "note": (valu or {}).get("note")}
    return res


def quotient_measure(args, dev, torch, world, dist):
    """The zkEVM-shaped constraint quotient (step42ns, starks.cpp:241) at its
    real domain, 2^24 rows: the full-size step42ns-shaped program (20 K ops,
    fork-9 memory map, 1,567 section columns in HBM) through the compiled
    segment kernels (csrc/zxp_segment.cpp).  Reported beside the config-4
    proof, whose own quotient is a small synthetic program."""
    import argparse as _ap
    import zkgpu
    a = _ap.Namespace(**vars(args))
    a.s42_scale, a.s42_jit, a.log_n = 1.0, True, 23
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED)
    step, s42 = step42ns_setup(a, dev, torch, g)
    elapsed, kernels = timed(step, args.s42_steps, 1, world, dist, torch)
    segs = {k: v for k, v in kernels.items() if k.startswith("k_zxp_jit")}
    dev_ms = sum(v[1] for v in segs.values()) / args.s42_steps
    roof = step42ns_roofline(s42, kernels, args.s42_steps)
    res = {"value": round(s42["rows"] * args.s42_steps / elapsed / 1e6, 3), "unit": "Mrow/s",
           "s_per_pass": round(elapsed / args.s42_steps, 4), "device_ms_per_pass": round(dev_ms, 3),
           "rows": s42["rows"], "n_ops": s42["n_ops"], "segments": len(segs),
           "segment_ms": [round(segs[k][1] / segs[k][0], 3) for k in sorted(segs)],
           "what": "step42ns-shaped synthetic program (zkgpu/synthetic_bytecode.py seed 1, the reference step42ns's "
                   "opcode histogram / temporaries / fork-9 map, tests/golden/zkevm_bytecode_shape.json) -> product "
                   "converter -> ZXP compile -> segment kernels; 2^24-row extended domain, sections resident in HBM; "
                   "parity: tests/test_gpu_full_parity.py (these segment kernels at the 2^24-row domain on ~1,000 "
                   "sampled rows, incl. the wrap rows, vs the oracle's case-table interpreter)"}
    f, d, why = _stamped("*_s42_pmc.json", "zxp")
    if roof is not None:
        roof["traffic_stamp"] = why
    if roof is not None and d and d.get("hbm_bytes_per_step"):
        roof["traffic"] = d["hbm_bytes_per_step"]
        roof["traffic_ratio"] = round(d["hbm_bytes_per_step"] / roof["alg_bytes_per_launch"], 2)
        roof["traffic_source"] = os.path.basename(f)
        roof["traffic_note"] = ("PMC HBM bytes per pass (2 x FETCH_SIZE + WRITE_SIZE): %.0f vector-memory reads per "
                                "row (column values, carries, limb-chunk prefetch; SQ_INSTS_VMEM_RD x 64 / rows) "
                                "against %d distinct column reads -- the program re-reads columns the registers "
                                "cannot hold (DESIGN.md 3.4)"
                                % (d["per_step"].get("SQ_INSTS_VMEM_RD", 0) * 64 / s42["rows"], s42["cols_read"]))
        roof["hbm_frac_measured_traffic"] = round(d["hbm_bytes_per_step"] / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        valu = d["per_step"].get("SQ_INSTS_VALU")
        if valu:
            rate = valu / (dev_ms * 1e-3)
            res["valu"] = {"wave_instr_per_pass": valu, "achieved": round(rate / 1e9, 1), "peak": 978.0,
                           "unit": "G wave-instr/s", "frac": round(rate / 978e9, 4),
                           "peak_model": "mix-weighted issue peak of the field-arithmetic kernels (DESIGN.md 3)",
                           "source": os.path.basename(f), "stamp": why}
    res["roofline"] = roof
    for t in s42["tensors"].values():
        del t
    s42.clear()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def handoff_pipelined(gs, s_per_proof, proofs=3):
    """Back-to-back proofs with the trace handed over from host memory:
    serial (set_cm1, then prove) against pipelined (set_cm1_async of the
    next proof's trace while the current one proves: the loader thread's
    PCIe copies and transposes run beside the proof's kernels,
    include/zkgpu_stark.h).  The trace is the instance's own witness read back
    (get_cm1), so the lookups hold."""
    rows = gs.get_cm1()
    res = {"bytes": int(rows.nbytes), "proofs": proofs}
    gs.set_cm1(rows)
    gs.prove_raw()  # warm
    t0 = time.perf_counter()
    for _ in range(proofs):
        gs.set_cm1(rows)
        gs.prove_raw()
    res["serial_s_per_proof"] = round((time.perf_counter() - t0) / proofs, 4)
    gs.set_cm1_async(rows)
    gs.prove_raw()  # warm: the loader's buffers
    t0 = time.perf_counter()
    for _ in range(proofs):
        gs.set_cm1_async(rows)
        gs.prove_raw()
    res["pipelined_s_per_proof"] = round((time.perf_counter() - t0) / proofs, 4)
    res["resident_s_per_proof"] = round(s_per_proof, 4)
    del rows
    return res


def handoff_measure(n, C, dev, torch, zkgpu, s_per_proof):
    """The drop-in boundary hands the committed trace over in HOST memory
    (zkevmCmPols file / executor buffer, row-major, commit_pols.hpp:18):
    time its upload into the device column-major section with the streamed
    loader (zkgpu_load_rows_dev: block H2D on a copy stream overlapped with
    the transposes), pageable and page-locked.  Reported beside the proof
    rate, never as `value` (the timed proof starts with the trace in HBM)."""
    import numpy as np
    rows = np.empty((n, C), np.uint64)
    rows.fill(1)  # touch every page before timing
    cols = torch.empty((C, n), dtype=torch.int64, device=dev)
    res = {"bytes": int(rows.nbytes), "what": "cm1 %d rows x %d cols, host row-major -> device column-major "
           "(zkgpu_load_rows_dev)" % (n, C)}
    for key, reg in (("pageable", False), ("registered", True)):
        best = None
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            zkgpu.load_rows_dev(cols, n, rows, register_host=reg)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        res[key] = {"ms": round(best * 1e3, 2), "GB/s": round(rows.nbytes / best / 1e9, 1)}
    up = min(res["pageable"]["ms"], res["registered"]["ms"]) * 1e-3
    res["s_per_proof_incl_upload"] = round(s_per_proof + up, 4)
    del rows, cols
    return res


def shm_outbox_bytes(inst, args, world):
    """Outbox of the host-staged exchange (bytes per rank and exchange): the
    largest message set a rank posts is a commit's return of its column share
    of the widest section, (W-1)/W of C 2N / W words, or its n-domain block
    (W-1)/W of C N / W words; with a quarter of margin, at least 256 MiB."""
    n = 1 << args.log_n
    widest = max(inst.n_cm1, inst.n_cm2, inst.n_cm3, inst.n_cm4, inst.n_const)
    share = -(-widest // world)
    words = max(share * (n << args.blowup_bits), widest * (n // world))
    return max(256 << 20, int(words * 8 * (world - 1) / world * 1.25))


def _coll_dev(dist):
    """device of the small tensors the bench's own collectives carry"""
    return "cpu" if dist.get_backend() == "gloo" else "cuda"


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def sharded_children(args, world, rank, local, dist, torch):
    """configs[4]: ONE proof over all ranks (zkgpu_stark_create_sharded, RCCL
    over xGMI), measured by child processes -- one per rank, on the rank's
    GPU, with their own rendezvous -- so that a failure there (the RCCL path
    has never run between GPUs on the builder's one-GPU lease) cannot take
    the replica measurement above with it: a child that fails or outlives
    --sharded-timeout is killed and reported.  Runs: the config-4 instance at
    every world size, and the fork-9 widths (751/168/408/6): 2^23 rows from
    W = 4 (190 GB per rank; 120 GB at W = 8), 2^22 rows on 1-2 ranks.  If the
    config-4 run over RCCL fails at N > 1, it runs again over the host-staged
    exchange (zkgpu_comm_host through /dev/shm), which then carries the
    headline with the line saying so, and the fork-9 runs are skipped.
    Returns rank 0's summary."""
    # fork-9 widths at 2^23 rows: on one GPU the single-GPU prover under the
    # lean HBM plan (271 GB; the row-sharded prover at W = 1 would hold every
    # section: 419 GB); from W = 2 the row-sharded prover (W = 2: 313 GB per
    # rank with the default LDE batches, 294 GB with the 32-column batches
    # create_sharded then picks; W = 4: 195 GB; W = 8: 132 GB).  If a W = 2
    # run at 2^23 fails, it runs again at 2^22 (and says so).
    single = world == 1  # the fork-9 runs through `--workload stark` (one GPU, AUTO plan -> lean)
    runs = [("config4", [], False), ("fork9", ["--fork9"], single), ("fork9_zkevm_shaped", ["--zkevm-shaped"], single)]
    out = {}
    for name, extra, one_gpu in runs:
        ok, rec = _sharded_child(args, world, rank, local, dist, torch, extra, "rccl", one_gpu)
        if not ok and name != "config4" and world == 2 and args.log_n > 22:
            ok, rec2 = _sharded_child(args, world, rank, local, dist, torch, extra + ["--log-n", "22"], "rccl", one_gpu)
            if rank == 0:
                rec = dict(rec2, run_at_2p23=rec) if ok else {"error": "2^23 and 2^22 runs failed", "run_at_2p23": rec,
                                                              "run_at_2p22": rec2}
        if rank == 0:
            out[name] = rec
        if ok:
            continue
        if name == "config4" and world > 1:
            # the RCCL run failed: the headline one-proof run again over the
            # host-staged exchange -- slower, but a real proof over the N GPUs
            ok2, rec2 = _sharded_child(args, world, rank, local, dist, torch, extra, "shm")
            if rank == 0:
                out[name] = dict(rec2, rccl_run=rec) if ok2 else {"error": "RCCL and host-staged runs failed",
                                                                  "rccl_run": rec, "shm_run": rec2}
                if ok2:
                    out[name]["exchange"] = "host shared memory (zkgpu_comm_host): the RCCL run failed"
        # the same code path again would fail the same way: no more runs
        if rank == 0:
            for later, _, _ in runs[runs.index((name, extra, one_gpu)) + 1:]:
                out[later] = {"error": "skipped after the failed %s run" % name}
        break
    return out if rank == 0 else None


def _sharded_child(args, world, rank, local, dist, torch, extra, comm, one_gpu=False):
    """One `--workload stark-sharded` run as a child process per rank (own
    rendezvous, --sharded-timeout); one_gpu (world 1): `--workload stark`, the
    single-GPU prover.  Returns (every rank's child succeeded, rank 0's
    record)."""
    import signal
    import subprocess
    port = _free_port() if rank == 0 else 0
    if world > 1:
        t = torch.tensor([port], dtype=torch.int64, device=_coll_dev(dist))
        dist.broadcast(t, 0)
        port = int(t.item())
    # ZKGPU_RUN_ID: the tag the host-staged exchange's ranks match their shared
    # segment on (host/comm_host.hpp; by default the launcher's pid, but each
    # rank's child here has its own parent)
    env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(local), WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ZKGPU_RUN_ID="bench-%d" % port)
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(world), "--workload",
           "stark" if one_gpu else "stark-sharded", "--steps", "3", "--warmup", "1", "--no-cpu", "--log-n",
           str(args.log_n), "--blowup-bits", str(args.blowup_bits), "--ncols", str(args.ncols), "--queries",
           str(args.queries), "--comm", comm] + extra  # (a later --log-n wins)
    if one_gpu:
        cmd += ["--no-lde", "--no-handoff", "--no-s42", "--no-sharded"]
    t0 = time.time()
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        so, se = p.communicate(timeout=args.sharded_timeout)
        rc = p.returncode
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        so, se = p.communicate()
        rc = "timeout"
    line = next((ln for ln in reversed(so.splitlines()) if ln.startswith('{"metric"')), None)
    mine = rc == 0 and (line is not None or rank != 0)
    if world > 1:  # every rank learns whether any child failed
        f = torch.tensor([0 if mine else 1], dtype=torch.int64, device=_coll_dev(dist))
        dist.all_reduce(f)
        ok = int(f.item()) == 0
    else:
        ok = mine
    if rank != 0:
        return ok, None
    if not mine:
        return ok, {"error": "exit %s" % rc, "comm": comm, "stderr_tail": se[-600:],
                    "wall_s": round(time.time() - t0, 1)}
    if not ok:
        return ok, {"error": "another rank's child failed", "comm": comm, "wall_s": round(time.time() - t0, 1)}
    d = json.loads(line)
    st = d.get("stages_ms") or {}
    rec = {"value": d["value"], "unit": d["unit"], "n_gpus": d["n_gpus"], "ms_per_step": d["ms_per_step"],
           "scaling": "strong", "workload": d["config"]["workload"], "log_n": d["config"]["log_n"],
           "prover": "single-GPU (zkgpu_stark_create)" if one_gpu else "row-sharded (zkgpu_stark_create_sharded)",
           "exchange_ms": round(sum(v for k, v in st.items() if "EXCHANGE" in k and not k.startswith("COUNT_")), 3),
           "stages_ms": {k: v for k, v in st.items() if not k.startswith("COUNT_COMM")},
           "wall_s": round(time.time() - t0, 1)}
    if d.get("comm"):
        rec["comm"] = d["comm"]
    return ok, rec


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) started without a launcher (no WORLD_SIZE):
    start N rank processes of this same command line -- RANK = LOCAL_RANK = i,
    WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free MASTER_PORT, as
    torch.distributed.run would -- and return the exit status.  Runs before
    anything here touches a GPU (no torch import in this process).  Rank 0's
    stdout is this process's stdout, so its JSON line is the line.  If a rank
    fails, the others get 60 s to finish and are then killed (a rank waiting in
    a collective for a dead peer never returns); the first failure's status is
    the result."""
    import signal
    import subprocess
    n = args.gpus
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
        raise SystemExit(128 + sig)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    status, deadline = 0, None
    while any(p.poll() is None for p in procs):
        for p in procs:
            rc = p.poll()
            if rc not in (None, 0) and status == 0:
                status = rc if rc > 0 else 128 - rc
                deadline = time.time() + 60
                sys.stderr.write("bench.py: rank %d exited with %s\n" % (procs.index(p), rc))
        if deadline is not None and time.time() > deadline:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    for i, p in enumerate(procs):
        if p.returncode and status == 0:
            status = p.returncode if p.returncode > 0 else 128 - p.returncode
            sys.stderr.write("bench.py: rank %d exited with %s\n" % (i, p.returncode))
    return status


def world_of(args):
    """(world, rank, local rank) this process runs as.  --gpus N must agree
    with the world a launcher (torch.distributed.run) put it in: a driver
    that asks for N GPUs never gets a line measured on another number."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d, but this process joined a world of %d ranks (WORLD_SIZE)"
                         % (args.gpus, world))
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def comm_summary(stages, world):
    """The C++ sharded prover's own account of its exchanges in the last proof
    (COUNT_COMM_* beside its stage timers): the world its communicator was
    created with and the bytes this rank (rank 0) sent."""
    if "COUNT_COMM_WORLD" not in stages:
        return None
    n = int(stages.get("COUNT_COMM_EXCHANGES", 0))
    sent = stages.get("COUNT_COMM_BYTES_SENT", 0.0)
    res = {"comm_world": int(stages["COUNT_COMM_WORLD"]), "exchanges_per_proof": n,
           "rank0_bytes_sent_per_proof": int(sent),
           "rank0_bytes_sent_per_exchange": int(sent / n) if n else 0,
           "rank0_largest_exchange_bytes": int(stages.get("COUNT_COMM_MAX_BYTES_SENT", 0)),
           "max_ops_per_exchange": int(stages.get("COUNT_COMM_MAX_OPS", 0))}
    # the device time inside the exchanges (stream marks around each one: the
    # transfers plus any wait for a slower peer) -> the achieved egress rate
    # of rank 0, against its W - 1 xGMI links (~153 GB/s each, 7 per MI355X)
    xms = stages.get("COUNT_COMM_EXCHANGE_MS")
    if xms:
        res["exchange_ms_per_proof"] = round(xms, 3)
        res["achieved_GBps"] = round(sent / (xms * 1e-3) / 1e9, 1)
        big = stages.get("COUNT_COMM_LARGEST_EXCHANGE_MS")
        if big:
            res["largest_exchange_ms"] = round(big, 3)
            res["largest_exchange_GBps"] = round(res["rank0_largest_exchange_bytes"] / (big * 1e-3) / 1e9, 1)
        res["link_peak_GBps"] = round(153.0 * (world - 1), 1)
        res["link_peak_note"] = "(W - 1) xGMI links x ~153 GB/s per direction (task brief figure; 7 links per GPU)"
    if res["comm_world"] != world:
        raise SystemExit("bench.py: the prover's communicator has world %d, the job %d" % (res["comm_world"], world))
    return res


def cpu_full_main(args):
    """Time the reference's CPU path restated (cpuref kernels under the
    oracle's orchestration) once at the full config-4 size (rank 0, no GPU)."""
    threads = _threads()
    inst = stark_instance(args.log_n, args.blowup_bits, args.ncols, args.queries)
    dt = _cpu_prove(inst, True)
    res = {"value": round(dt, 3), "unit": "s/proof", "cores": threads, "kind": "restated-reference-AVX2",
           "what": REF_NOTE, "sample": "the whole config-4 proof at 2^%d rows, %d threads (%s)"
                                       % (args.log_n, threads, _cpu_model()),
           "note": "full-size run: bench.py --cpu-full (the default bench quotes it as cpu_baseline.full_size)"}
    print(json.dumps(res), flush=True)


def main():
    args = parse()
    if args.cpu_full:
        return cpu_full_main(args)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world, rank, local = world_of(args)
    if args.rank_probe:  # launcher check (tests/test_bench_launch.py): no GPU, no torch
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                        "MASTER_PORT")}), flush=True)
        if os.environ.get("ZKGPU_BENCH_PROBE_FAIL") == str(rank):
            sys.exit(3)  # the launcher's failure path
        return
    import torch
    import torch.distributed as dist
    import zkgpu

    # ZKGPU_BENCH_SHARE_GPU=1 (tests only, tests/test_gpu_bench_ranks.py):
    # every rank on device 0 with a gloo group -- the multi-rank bench on the
    # one-GPU test box, where RCCL refuses two ranks on one device
    share = os.environ.get("ZKGPU_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    if world > 1:
        dist.init_process_group("gloo" if share else "nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    zkgpu.init(local)
    stream = torch.cuda.current_stream()
    zkgpu.set_stream(stream)

    n = 1 << args.log_n
    ne = n << args.blowup_bits
    C = args.ncols
    res = {"metric": METRIC}
    gs = inst = None
    prepare = None
    lean = False
    sharded = None
    lde = roof = handoff = quotient = None
    if args.workload == "lde":
        lde, roof = lde_measure(args, dev, torch, world, dist)
        elapsed = lde["ms_per_lde"] * 1e-3 * args.steps
        value, unit, hib = lde["value"], "Gelem/s", True
        kernels = None
    else:
        g = torch.Generator(device=dev)
        g.manual_seed(0x5EED + rank)
        if args.workload == "stark":
            from zkgpu.stark import GpuStark
            inst = stark_instance(args.log_n, args.blowup_bits, C, args.queries, _kind(args))
            gs = GpuStark(inst)  # setup: constants, constant LDE + tree (untimed; files in the reference)
            gs.witness()         # executor stand-in: committed trace cm1 in HBM (untimed)
            if gs.memory_mode() == "lean":
                # the lean HBM plan (include/zkgpu_stark.h) extends the trace in
                # place: every proof gets a fresh one, loaded outside its timing
                prepare = gs.witness

            def step():
                gs.prove_raw()
        elif args.workload == "stark-sharded":
            # the C++ row-sharded prover (host/sharded_starks.hpp) over RCCL,
            # or over host shared memory (--comm shm: outboxes sized for the
            # instance's largest exchange, named after this run's rendezvous)
            from zkgpu.stark import GpuStark, RcclComm, ShmComm
            inst = stark_instance(args.log_n, args.blowup_bits, C, args.queries, _kind(args))
            if args.comm == "shm":
                comm = ShmComm("/zkgpu_bench_%s" % os.environ.get("MASTER_PORT", "0"), world, rank,
                               shm_outbox_bytes(inst, args, world))
            else:
                comm = RcclComm()
            gs = GpuStark(inst, comm=comm)
            gs.witness()

            def step():
                gs.prove_raw()
        elif args.workload == "step42ns":
            step, s42 = step42ns_setup(args, dev, torch, g)
        else:  # merkle
            src = torch.randint(0, 2**63 - 1, (C, n), dtype=torch.int64, device=dev, generator=g)
            nodes = torch.empty(zkgpu.merkle_num_elements(n), dtype=torch.int64, device=dev)

            def step():
                zkgpu.merkletree_dev(nodes, src, n, C, n)
        elapsed, kernels = timed(step, args.steps, args.warmup, world, dist, torch, prepare)
        elapsed = max_over_ranks(elapsed, world, dist, torch, dev)
        if args.workload in ("stark", "stark-sharded"):
            total = (world if args.workload == "stark" else 1) * args.steps
            value, unit, hib = elapsed / total, "s/proof", False
        elif args.workload == "step42ns":
            value, unit, hib = s42["rows"] * world * args.steps / elapsed / 1e6, "Mrow/s", True
            roof = step42ns_roofline(s42, kernels, args.steps)
        else:
            value, unit, hib = n * C * world * args.steps / elapsed / 1e9, "Gelem/s", True
        stages = gs.timers() if gs is not None else None
        lean = prepare is not None
        if lean:
            # a lean prover holds what the HBM had to spare (its kept columns):
            # release it (and the bound witness method holding it) before the
            # LDE line allocates
            gs = prepare = step = None
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        if args.workload == "stark" and not args.no_lde:
            lde, roof = lde_measure(args, dev, torch, world, dist)
        if args.workload == "stark" and world == 1 and not args.no_handoff and not lean:
            handoff = handoff_measure(n, inst.n_cm1, dev, torch, zkgpu, value)
            handoff["pipelined"] = handoff_pipelined(gs, value)
        if args.workload == "stark" and world == 1 and args.log_n == 23 and not args.no_s42:
            gs = None  # the config-4 instance's HBM back before the 200 GB of fork-9-width sections
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            quotient = quotient_measure(args, dev, torch, world, dist)
        if args.workload == "stark" and not args.no_sharded:
            gs = None  # the replica prover's HBM back for the children
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            zkgpu.release()  # and the library's workspaces (this process is done with the GPU)
            sharded = sharded_children(args, world, rank, local, dist, torch)

    # N > 1: the headline is ONE config-4 proof over all ranks (configs[4],
    # strong scaling against the N = 1 line's single-GPU proof); the replica
    # throughput above moves to a side block.  If the one-proof run failed,
    # the replicas stay the value and the line says so.
    replicas = None
    scaling = "strong" if args.workload == "stark-sharded" else "weak"
    if rank == 0 and args.workload == "stark" and world > 1:
        replicas = {"value": round(value, 4), "unit": unit, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                    "meaning": "one independent config-4 proof per GPU (replicas): wall seconds per proof over the "
                               "whole job", "steps": args.steps}
        one = (sharded or {}).get("config4") or {}
        if one.get("value"):
            value, elapsed = one["value"], one["ms_per_step"] * 1e-3 * args.steps
            scaling = "strong"
            replicas["note"] = "the headline value is sharded_one_proof.config4"
        else:
            replicas["note"] = ("the one-proof-over-%d-ranks run failed (sharded_one_proof.config4): the value is the "
                                "replica throughput" % world)
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            if args.workload == "stark":
                cpu = cpu_baseline_stark(min(args.cpu_sample_bits, args.log_n), args.blowup_bits, C, args.queries)
                full = cpu_full_size_record()
                if full and full.get("value"):
                    key = "full_size" if full.get("kind") == cpu["kind"] else "port_full_size"
                    cpu[key] = full
                    cpu[key + "_vs_gpu"] = round(full["value"] / value, 1)
                if not args.no_cpu_zkevm:
                    z = cpu_baseline_zkevm(16, args.queries)
                    g = ((sharded or {}).get("fork9_zkevm_shaped") or {})
                    if g.get("value"):
                        rows = 1 << g.get("log_n", args.log_n)
                        z["gpu_same_instance"] = {"s_per_proof": g["value"], "rows": rows,
                                                  "source": "sharded_one_proof.fork9_zkevm_shaped (1 GPU)"}
                        z["per_row_ratio"] = round((z["value"] / z["rows"]) / (g["value"] / rows), 1)
                        z["per_row_ratio_note"] = ("CPU seconds per trace row at 2^16 / GPU seconds per row at 2^%d: a "
                                                   "throughput ratio of the same proof, not an extrapolated full-size "
                                                   "time (the CPU's per-row cost still falls with size: FRI and queries "
                                                   "are a fixed cost)" % g.get("log_n", args.log_n))
                    cpu["zkevm_shaped"] = z
            elif args.workload == "lde":
                cpu = cpu_baseline_lde(args.log_n, args.blowup_bits, args.cpu_sample_cols)
            elif args.workload == "merkle":
                cpu = cpu_baseline_merkle(args.log_n, C)
        if args.workload == "stark":
            kind = _kind(args)
            workload = ("full STARK proof (genProof stages 1-5 + FRI + queries, starks.cpp:9-404), %s: 2^%d trace, "
                        "blowup 2^%d, cm1/cm2/cm3/cm4 = %d/%d/%d/%d, %d constants, %d tmpExp, 2 plookups, post-Z step3, "
                        "FRI steps %s, %d queries, %d evaluations; trace resident in HBM; one independent proof per GPU"
                        "; HBM plan: %s"
                        % ("the zkEVM-shaped instance (fork-9 widths + the five zkEVM-shaped expression programs, "
                           "zkgpu/zkevm_shaped.py)" if kind == "zkevm" else "the fork-9-width synthetic instance"
                           if kind else "synthetic config-4 instance", args.log_n, args.blowup_bits, inst.n_cm1,
                           inst.n_cm2, inst.n_cm3, inst.n_cm4, inst.n_const, inst.n_tmp, inst.fri_steps, args.queries,
                           len(inst.evmap),
                           "lean (sections share one arena by lifetime, cm1 / cm3 extended in place; the proof consumes "
                           "its trace, so each timed proof gets a fresh one from the executor stand-in outside its "
                           "own barrier + synchronize bracket)" if lean else "resident"))
            one = (sharded or {}).get("config4") or {}
            parallelism = ("replicas x%d (one independent proof per GPU)" % world if world == 1 or scaling == "weak"
                           else "ONE proof row-sharded x%d (sharded_one_proof.config4: C++ prover, %s exchange of "
                                "packed column/row blocks per commit); replicas in the `replicas` block"
                                % (world, "host shared memory (the RCCL run failed)" if one.get("exchange") else "RCCL"))
        elif args.workload == "stark-sharded":
            workload = ("ONE %s STARK proof (2^%d trace, cm1/cm2/cm3/cm4 = %d/%d/%d/%d, %d constants, %d queries) "
                        "row-sharded over %d rank(s): n and 2n domains by rows, NTT-transpose all-to-all per commit"
                        % ("zkEVM-shaped (fork-9 widths + the five zkEVM-shaped expression programs, "
                           "zkgpu/zkevm_shaped.py)" if args.zkevm_shaped else
                           "fork-9-width" if args.fork9 else "config-4", args.log_n, inst.n_cm1, inst.n_cm2,
                           inst.n_cm3, inst.n_cm4, inst.n_const, args.queries, world))
            parallelism = ("one proof, n and 2n domains row-sharded x%d (C++ prover, host/sharded_starks.hpp): per "
                           "exchange one RCCL send + one receive per peer (packed column/row blocks with halos per "
                           "commit, quotient split by column owners, f row gather)" % world)
        elif args.workload == "lde":
            workload = ("LDE 2^%d -> 2^%d rows x %d cols per GPU (extendPol, starks.cpp:53), column-major in HBM"
                        % (args.log_n, args.log_n + args.blowup_bits, C))
            parallelism = "column-sharded x%d (no data-path collective)" % world
        elif args.workload == "step42ns":
            workload = ("Steps::step42ns_parser_first (constraint quotient, starks.cpp:241) over the 2^%d-row "
                        "extended domain: a synthetic program with the reference step42ns bytecode's shape (%d ops = "
                        "%g x the opcode histogram, fork-9 memory map, next-row reads; tests/golden/"
                        "zkevm_bytecode_shape.json) through the product converter and the %s; sections resident in HBM"
                        % (s42["log_dom"], s42["n_ops"], args.s42_scale,
                           "compiled expression kernel" if args.s42_jit else "expression interpreter"))
            parallelism = "replicas x%d" % world
        else:
            workload = ("Poseidon-GL Merkle tree over 2^%d rows x %d cols per GPU (merkelize, merkleTreeGL.cpp:37-44)"
                        % (args.log_n, C))
            parallelism = "replicas x%d" % world
        res.update({
            "value": round(value, 4),
            "unit": unit,
            "value_meaning": ("wall seconds per proof, whole job" if unit == "s/proof"
                              else "elements per second, all GPUs"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": hib,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u64 (Goldilocks) + F_p^3" if args.workload.startswith("stark") else "u64 (Goldilocks)",
            "data": "synthetic (uniform canonical Goldilocks; trace from the instance PRNG / torch generator seed "
                    "0x5EED+rank)",
            "config": {"workload": workload, "log_n": args.log_n, "blowup_bits": args.blowup_bits,
                       "ncols_per_gpu": C, "parallelism": parallelism},
        })
        if lde is not None and args.workload != "lde":
            res["lde"] = lde
        if roof is not None:
            res["roofline"] = roof
        if handoff is not None:
            res["handoff"] = handoff
        if quotient is not None:
            res["quotient_zkevm_shaped"] = quotient
        if sharded is not None:
            res["sharded_one_proof"] = sharded
            ns = sharded.get("fork9_zkevm_shaped") or {}
            if ns.get("value"):
                # the north-star instance (BASELINE.json north_star: the 2^23-row
                # zkEVM trace), surfaced beside the config-4 headline
                res["north_star"] = {
                    "value": ns["value"], "unit": ns["unit"], "n_gpus": ns["n_gpus"], "log_n": ns.get("log_n"),
                    "instance": "fork-9 widths (751/168/408/6 committed, 234 constants) + the five zkEVM-shaped "
                                "expression programs (zkgpu/zkevm_shaped.py)",
                    "prover": ns.get("prover"),
                    "hbm_plan": "lean (one GPU)" if world == 1 else "row-sharded",
                    "verified_by": "tests/test_gpu_verify_full.py (verifier replay of the GPU's 2^23 proof: transcript, "
                                   "every Merkle path, every FRI fold, the FRI polynomial at the query rows)",
                    "source": "sharded_one_proof.fork9_zkevm_shaped"}
        if replicas is not None:
            res["replicas"] = replicas
            one = (sharded or {}).get("config4") or {}
            if one.get("comm") and scaling == "strong":
                res["comm"] = one["comm"]  # the headline proof's exchanges (C++ prover's count)
        if kernels is not None:
            res["kernels"] = kernel_table(kernels)
            if args.workload == "stark" and args.log_n == 23 and C == 100:
                dom = max(kernels, key=lambda k: kernels[k][1])
                res["dominant_kernel"] = {"kernel": dom, "share_of_device_time": round(
                    kernels[dom][1] / sum(v[1] for v in kernels.values()), 3)}
                if "k_leaves_cols" in kernels:
                    v = kernels["k_leaves_cols"]
                    res["valu"] = stark_valu("k_leaves_cols", v[1] / args.steps, int(round(v[0] / args.steps)))
                    res["leaves"] = leaves_line(inst, args, v)
                    res["roofline_dominant"] = dominant_roofline(inst, args, v, res["valu"])
            if args.workload in ("stark", "stark-sharded") and stages:
                res["stages_ms"] = {k: round(v, 3) for k, v in stages.items()}
                comm = comm_summary(stages, world)
                if comm:
                    res["comm"] = comm
        res["cpu_baseline"] = cpu
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
