#!/bin/bash
# full-size step42ns-shaped quotient at 2^24 rows under several JIT variants
# (env), one bench process each; kernels prebuilt into the jitcache
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s42var
i=0
while read -r v; do
    echo "== $v" > gpurun_out/s42var/v$i.log
    env $v timeout -k 10 120 python -u bench.py --workload step42ns --s42-jit --s42-scale 1 --steps 3 --warmup 1 \
        >> gpurun_out/s42var/v$i.log 2>&1 || { echo "variant $i failed"; exit 1; }
    i=$((i+1))
done <<'VARS'
ZKGPU_ZXP_JIT_ROWS=1 ZKGPU_ZXP_JIT_DOTLOOP=100000 ZKGPU_ZXP_JIT_WAVES=4
ZKGPU_ZXP_JIT_ROWS=1 ZKGPU_ZXP_JIT_DOTLOOP=100000 ZKGPU_ZXP_JIT_WAVES=3
ZKGPU_ZXP_JIT_ROWS=2 ZKGPU_ZXP_JIT_DOTLOOP=100000 ZKGPU_ZXP_JIT_WAVES=2
ZKGPU_ZXP_JIT_ROWS=1 ZKGPU_ZXP_JIT_DOTLOOP=100000
ZKGPU_ZXP_JIT_ROWS=2 ZKGPU_ZXP_JIT_DOTLOOP=100000
ZKGPU_ZXP_JIT_ROWS=2
VARS
