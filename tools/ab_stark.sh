#!/bin/bash
# A/B of env-selected kernel variants on the config-4 STARK proof (bench.py
# --workload stark, no side measurements): one bench process per variant,
# baseline first and last; prints s/proof and the expression-stage timers.
# The variants' code objects must be in the JIT cache (prebuilt on the CPU).
# AB_BENCH_ARGS: extra bench.py arguments (e.g. "--zkevm-shaped --log-n 22").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
    local tag=$1
    shift
    env "$@" timeout -k 10 300 python bench.py --workload stark --no-lde --no-s42 --no-sharded --no-cpu --no-handoff \
        --steps 3 --warmup 1 ${AB_BENCH_ARGS:-} > gpurun_out/ab_stark.json 2> gpurun_out/ab_stark.err
    local rc=$?
    [ $rc -eq 0 ] || { echo "[ab_stark] $tag rc=$rc"; tail -3 gpurun_out/ab_stark.err; exit $rc; }
    python3 -c "
import json, sys
d = json.load(open('gpurun_out/ab_stark.json'))
s = d['stages_ms']
print('[ab_stark] %-44s %.4f s  q %.2f  fri %.2f  e2 %.2f  e3 %.2f' % (sys.argv[1], d['value'], s['STARK_STEP_4_CALCULATE_EXPS_2NS'],
      s['STARK_STEP_5_CALCULATE_EXPS'], s['STARK_STEP_2_CALCULATE_EXPS'], s['STARK_STEP_3_CALCULATE_EXPS']))" "$tag" | tee -a gpurun_out/ab_stark.log
}
run baseline ZKGPU_AB=0
for v in "$@"; do
    run "$v" $v
done
run baseline ZKGPU_AB=0
