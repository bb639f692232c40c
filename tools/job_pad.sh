#!/bin/bash
# quotient at 2^24 rows with padded column strides (L2 set aliasing A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pad
mkdir -p $O
for pad in 0 64 72 136 520 0; do
  ZKGPU_S42_PAD=$pad timeout -k 10 200 python bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 --warmup 1 > $O/p$pad.json 2> $O/p$pad.err || exit $?
  python -c "import json; d=json.load(open('$O/p$pad.json')); print('pad $pad', d['value'], d['ms_per_step'])"
done
