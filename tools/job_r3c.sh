#!/bin/bash
# round 3: quotient segment occupancy A/B (2 / 3 / 4 waves per SIMD) with the reference's locality
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3c
mkdir -p $O
for w in 4 3 2; do
  ZKGPU_ZXP_SEG_WAVES=$w timeout -k 10 300 python bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 --warmup 1 > $O/w$w.json 2> $O/w$w.err || exit $?
  python -c "import json; d=json.load(open('$O/w$w.json')); print('waves $w', d['value'], d['ms_per_step'])"
done
