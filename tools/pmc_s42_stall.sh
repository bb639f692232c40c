#!/bin/bash
# Stall / issue counters of the zkEVM-shaped quotient segments (one step),
# three rocprofv3 --pmc passes, each its own process and time limit.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s42_stall${1:-}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 1 --warmup 0"
n=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_IFETCH SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_WAVES" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
    n=$((n + 1))
    timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-trace -d $O/p$n -o p --output-format csv -- $B > $O/p$n.log 2>&1
    rc=$?
    echo "[s42_stall] pass $n rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
