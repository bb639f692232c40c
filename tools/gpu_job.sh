#!/bin/bash
# GPU job runner for gpurun: each GPU step has its own time limit; the job
# stops at the first fault / abort / segfault / timeout (exit >= 124 or
# signal), but continues past an ordinary test failure (exit 1).
# Usage: tools/gpu_job.sh <step>...
#   steps: tests large smoke bench benchq instbench bwbench parser step42ns prof trace1 pmc cpufull merkle
#          zkevm northstar profns sharded
#   parametrised (replace the round-by-round one-off scripts):
#     pytest:<file>[,<file>...]   those test files (-x -v, 300 s per test)
#     benchargs:<tag>             python bench.py $BENCH_ARGS -> gpurun_out/bench_<tag>.json
#     ab:<tag>                    tools/ab_lib.sh <tag> $AB_ARGS (this tree's lib vs lib_ab)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() {
    local rc=$1 what=$2
    echo "[gpu_job] $what exit=$rc" | tee -a gpurun_out/job.log
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "[gpu_job] stopping after $what (rc=$rc)" | tee -a gpurun_out/job.log
        exit "$rc"
    fi
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
for step in "$@"; do
    case "$step" in
    tests)
        timeout -k 10 1200 $PYT tests -m gpu --deselect tests/test_gpu_large.py --deselect tests/test_gpu_config4.py \
            ${PYTEST_EXTRA:-} > gpurun_out/pytest_gpu.log 2>&1
        ok_or_stop $? "pytest -m gpu"
        tail -5 gpurun_out/pytest_gpu.log
        ;;
    large)
        timeout -k 10 900 $PYT tests/test_gpu_large.py tests/test_gpu_config4.py > gpurun_out/pytest_gpu_large.log 2>&1
        ok_or_stop $? "pytest large"
        tail -5 gpurun_out/pytest_gpu_large.log
        ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
        ok_or_stop $? "smoke"
        tail -3 gpurun_out/smoke.log
        ;;
    bench)
        timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
        ok_or_stop $? "bench"
        cat gpurun_out/bench.json
        ;;
    benchq)
        timeout -k 10 600 python bench.py --no-cpu > gpurun_out/benchq.json 2> gpurun_out/benchq.err
        ok_or_stop $? "bench (no cpu)"
        cat gpurun_out/benchq.json
        ;;
    instbench)
        timeout -k 10 120 build/instbench > gpurun_out/instbench.json 2> gpurun_out/instbench.err
        ok_or_stop $? "instbench"
        ;;
    bwbench)
        timeout -k 10 120 build/bwbench > gpurun_out/bwbench.json 2> gpurun_out/bwbench.err
        ok_or_stop $? "bwbench"
        cat gpurun_out/bwbench.json
        ;;
    parser)
        timeout -k 10 600 $PYT tests/test_gpu_parser.py > gpurun_out/pytest_parser.log 2>&1
        ok_or_stop $? "pytest parser"
        tail -5 gpurun_out/pytest_parser.log
        ;;
    cpufull)
        timeout -k 10 1000 python bench.py --cpu-full > gpurun_out/cpu_full_stark.json 2> gpurun_out/cpu_full.err
        ok_or_stop $? "cpu full-size oracle"
        cat gpurun_out/cpu_full_stark.json
        ;;
    prof)
        cd /tmp
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/gpurun_out/prof" -o run \
            --output-format csv -- python3 "$ROOTDIR/bench.py" --no-cpu \
            > "$ROOTDIR/gpurun_out/prof_bench.json" 2> "$ROOTDIR/gpurun_out/prof.err"
        rc=$?
        cd "$ROOTDIR"
        ok_or_stop $rc "rocprofv3 kernel-trace"
        ;;
    trace1)
        # per-dispatch kernel trace of one timed STARK proof (after one warmup proof)
        cd /tmp
        timeout -k 10 400 rocprofv3 --kernel-trace -d "$ROOTDIR/gpurun_out/trace1" -o run \
            --output-format csv -- python3 "$ROOTDIR/bench.py" --workload stark --no-cpu --no-lde --steps 1 --warmup 1 \
            > "$ROOTDIR/gpurun_out/trace1_bench.json" 2> "$ROOTDIR/gpurun_out/trace1.err"
        rc=$?
        cd "$ROOTDIR"
        ok_or_stop $rc "rocprofv3 kernel-trace (one proof)"
        ;;
    pmc)
        # every counter bench.py's ratios read, stamped (tools/pmc_round.sh -> profiles/${PMC_TAG}_*)
        bash tools/pmc_round.sh ${PMC_TAG:-r04} > gpurun_out/pmc_round.log 2>&1
        ok_or_stop $? "pmc round"
        tail -3 gpurun_out/pmc_round.log
        ;;
    step42ns)
        timeout -k 10 600 python bench.py --workload step42ns --no-cpu --steps 3 --warmup 1 \
            > gpurun_out/bench_step42ns.json 2> gpurun_out/bench_step42ns.err
        ok_or_stop $? "bench step42ns"
        cat gpurun_out/bench_step42ns.json
        ;;
    merkle)
        timeout -k 10 600 python bench.py --workload merkle --steps 3 --warmup 1 > gpurun_out/bench_merkle.json 2> gpurun_out/bench_merkle.err
        ok_or_stop $? "bench merkle"
        cat gpurun_out/bench_merkle.json
        ;;
    zkevm)
        timeout -k 10 300 python -u bench.py --workload stark --zkevm-shaped --log-n 22 --steps 3 --warmup 1 --no-cpu \
            --no-lde --no-handoff --no-s42 --no-sharded > gpurun_out/bench_zkevm.json 2> gpurun_out/bench_zkevm.err
        ok_or_stop $? "bench zkevm-shaped 2^22"
        cat gpurun_out/bench_zkevm.json
        ;;
    pytest:*)
        files=$(echo "${step#pytest:}" | tr ',' ' ')
        timeout -k 10 1100 $PYT $files > gpurun_out/pytest_files.log 2>&1
        ok_or_stop $? "pytest $files"
        tail -5 gpurun_out/pytest_files.log
        ;;
    benchargs:*)
        tag=${step#benchargs:}
        timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > "gpurun_out/bench_$tag.json" 2> "gpurun_out/bench_$tag.err"
        ok_or_stop $? "bench $tag (${BENCH_ARGS:-})"
        tail -c 1500 "gpurun_out/bench_$tag.json"
        ;;
    ab:*)
        bash tools/ab_lib.sh "${step#ab:}" ${AB_ARGS:-}
        ok_or_stop $? "A/B ${step#ab:}"
        ;;
    northstar)
        # the north-star instance: fork-9 widths + zkEVM-shaped programs, 2^23 rows, one GPU (lean HBM plan)
        timeout -k 10 400 python -u bench.py --workload stark --zkevm-shaped --log-n 23 --steps 3 --warmup 1 --no-cpu \
            --no-lde --no-handoff --no-s42 --no-sharded > gpurun_out/bench_northstar.json 2> gpurun_out/bench_northstar.err
        ok_or_stop $? "bench north star 2^23"
        tail -c 600 gpurun_out/bench_northstar.json
        ;;
    profns)
        cd /tmp
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/gpurun_out/prof_ns" -o run --output-format csv -- \
            python3 "$ROOTDIR/bench.py" --workload stark --zkevm-shaped --log-n 23 --steps 2 --warmup 1 --no-cpu --no-lde \
            --no-handoff --no-s42 --no-sharded > "$ROOTDIR/gpurun_out/prof_ns.json" 2> "$ROOTDIR/gpurun_out/prof_ns.err"
        rc=$?
        cd "$ROOTDIR"
        ok_or_stop $rc "rocprofv3 kernel-trace (north star)"
        ;;
    sharded)
        timeout -k 10 600 $PYT tests/test_gpu_sharded_cpp.py tests/test_gpu_zkevm_shaped.py > gpurun_out/pytest_sharded.log 2>&1
        ok_or_stop $? "pytest sharded stark gpu"
        tail -3 gpurun_out/pytest_sharded.log
        ;;
    *)
        echo "unknown step $step"
        ;;
    esac
done
echo "[gpu_job] done" | tee -a gpurun_out/job.log
