#!/bin/bash
# A/B of the run-time compiled expression kernels' generation options on the
# 2^23 STARK: s/proof and the quotient / FRI-polynomial stage times
# usage: tools/jit_ab.sh tag:VAR=val,VAR=val ...   (tag "default" = no override)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "${@:-default:ZKGPU_NOP=1}"; do
    tag=${spec%%:*}
    vars=${spec#*:}
    env ${vars//,/ } timeout -k 10 240 python bench.py --workload stark --no-cpu --no-lde --steps 3 --warmup 1 \
        > gpurun_out/jitab_$tag.json 2> gpurun_out/jitab_$tag.err || { echo "$tag failed"; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/jitab_$tag.json')); s=d['stages_ms']
print('$tag', d['value'], 'q', s['STARK_STEP_4_CALCULATE_EXPS_2NS'], 'f', s['STARK_STEP_5_CALCULATE_EXPS'], 's2', s['STARK_STEP_2_CALCULATE_EXPS'])"
done
