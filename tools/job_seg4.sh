#!/bin/bash
# config-4 STARK: expression programs as 1 / 2 / 3 segments (occupancy of the quotient)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/seg4
mkdir -p $O
for rep in 1 2; do
for s in def 2 3; do
  if [ $s = def ]; then unset ZKGPU_ZXP_SEGMENTS; else export ZKGPU_ZXP_SEGMENTS=$s; fi
  timeout -k 10 300 python bench.py --no-cpu --no-s42 --no-sharded --no-handoff --no-lde --steps 5 --warmup 2 > $O/s${s}_$rep.json 2> $O/s${s}_$rep.err || exit $?
  python -c "import json; d=json.load(open('$O/s${s}_$rep.json')); st=d['stages_ms']; print('$s rep $rep', d['value'], st['STARK_STEP_4_CALCULATE_EXPS_2NS'], st['STARK_STEP_5_CALCULATE_EXPS'], st['STARK_STEP_2_CALCULATE_EXPS'], st['STARK_STEP_3_CALCULATE_EXPS'])"
done
done
