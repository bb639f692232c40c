#!/bin/bash
# LDS column cache: HBM fetch and issue/wait counters of the zkEVM-shaped quotient, cache off / 12 / 16 slots
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/lcpmc
mkdir -p $O
B="python3 $R/bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 --warmup 1"
cd /tmp && export TMPDIR=/tmp
for v in 0 12 16; do
  export ZKGPU_ZXP_JIT_LCACHE=$v
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/l$v/p3 -o p --output-format csv -- $B > $O/l$v.p3.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -d $O/l$v/p1 -o p --output-format csv -- $B > $O/l$v.p1.log 2>&1 || exit $?
  python3 $R/tools/s42_pmc_summary.py $O/l$v $O/l$v.json 3 > /dev/null && python3 -c "
import json; d=json.load(open('$O/l$v.json')); print('lcache $v', 'HBM TB/step', round(d['hbm_bytes_per_step']/1e12, 3), {k: round(v/1e9, 2) for k, v in d['per_step'].items()})"
done
