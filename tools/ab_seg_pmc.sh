#!/bin/bash
# quotient segment variants: A/B timings, then FETCH/WRITE counters of baseline and one variant
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/abpmc
bash tools/ab_env.sh "ZKGPU_ZXP_SEG_AB=3,20,0" "ZKGPU_ZXP_SEG_AB=3,20,8" "ZKGPU_ZXP_SEG_AB=3,20,16" "ZKGPU_ZXP_SEG_AB=3,20,24" "ZKGPU_ZXP_SEG_AB=3,22,16" "ZKGPU_ZXP_SEG_AB=3,16,16" "ZKGPU_ZXP_SEG_AB=3,22,32" > gpurun_out/ab_env_run2.log 2>&1 || exit $?
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 2 --warmup 1"
for v in 0 3,20,16; do
  for c in FETCH_SIZE WRITE_SIZE; do
    if [ "$v" = 0 ]; then unset ZKGPU_ZXP_SEG_AB; else export ZKGPU_ZXP_SEG_AB=$v; fi
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/abpmc/${v}_$c -o p --output-format csv -- $B > $R/gpurun_out/abpmc/${v}_$c.log 2>&1
    rc=$?; echo "[abpmc] $v $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
