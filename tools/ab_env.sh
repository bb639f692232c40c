#!/bin/bash
# A/B of env-selected kernel variants on the zkEVM-shaped quotient (bench.py
# --workload step42ns --s42-jit): one bench process per variant, baseline
# first and last.  The variants' code objects must be in the JIT cache
# already (prebuilt on the CPU).  Usage: tools/ab_env.sh "ENV=V ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
    local tag=$1
    shift
    env "$@" timeout -k 10 240 python bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 \
        --warmup 1 > gpurun_out/ab_env.json 2> gpurun_out/ab_env.err
    local rc=$?
    [ $rc -eq 0 ] || { echo "[ab_env] $tag rc=$rc"; tail -3 gpurun_out/ab_env.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_env.json')); print('[ab_env] %-40s %8.2f Mrow/s  %8.2f ms' % (sys.argv[1], d['value'], d['roofline']['avg_launch_ms']))" "$tag" | tee -a gpurun_out/ab_env.log
}
run baseline ZKGPU_AB=0
for v in "$@"; do
    run "$v" $v
done
run baseline ZKGPU_AB=0
