#!/bin/bash
# compiled quotient kernel of the quarter-size step42ns-shaped program at 2^24
# rows for several basic-block sizes (ZKGPU_ZXP_JIT_BLOCK, source bytes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in "$@"; do
    ZKGPU_ZXP_JIT_BLOCK=$b timeout -k 10 300 python bench.py --workload step42ns --no-cpu --steps 3 --warmup 1 \
        --s42-scale 0.25 --s42-jit > gpurun_out/s42_b$b.json 2> gpurun_out/s42_b$b.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/s42_b$b.json'));print('block $b', d['value'], 'Mrow/s', d['ms_per_step'], 'ms')"
done
