#!/bin/bash
# Counters and kernel statistics bench.py's ratios come from, collected on the
# GPU box from ONE build of the tree, then summarised and stamped by
# tools/pmc_summary.py (zkgpu/stamp.py source hashes) into profiles/<tag>_*.
#   stats    rocprofv3 --kernel-trace --stats of the default bench command
#   stark    one config-4 proof: SQ (+ GRBM clock) / FETCH_SIZE / WRITE_SIZE passes
#   lde      configs[1] LDE: the same three passes
#   s42      the zkEVM-shaped quotient (step42ns-shaped program, 2^24 rows): the same
#   pb       the isolated permutation benchmark (build/poseidon_bench)
# Each rocprofv3 run is its own process with its own time limit; the script
# stops at the first failure.  Usage (GPU box): tools/pmc_round.sh <tag> [steps...]
set -u
TAG=$1
shift
STEPS=${*:-stats stark lde s42 pb}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
pass() {  # name, counters, command...
    local name=$1 ctr=$2
    shift 2
    timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d $O/$name -o p --output-format csv -- "$@" \
        > $O/$name.log 2>&1
    local rc=$?
    echo "[pmc_round] $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
for step in $STEPS; do
    case $step in
    stats)
        timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/stats -o p --output-format csv -- \
            python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-sharded > $O/stats_bench.json 2> $O/stats.log
        rc=$?; echo "[pmc_round] stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
        ;;
    stark)
        B="python3 $R/bench.py --workload stark --steps 1 --warmup 0 --no-cpu --no-lde --no-handoff --no-s42 --no-sharded"
        pass stark_sq "$SQ" $B
        pass stark_fetch FETCH_SIZE $B
        pass stark_write WRITE_SIZE $B
        ;;
    lde)
        B="python3 $R/bench.py --workload lde --steps 2 --warmup 1 --no-cpu"
        pass lde_sq "$SQ" $B
        pass lde_fetch FETCH_SIZE $B
        pass lde_write WRITE_SIZE $B
        ;;
    s42)
        B="python3 $R/bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 2 --warmup 1"
        pass s42_sq "$SQ" $B
        pass s42_fetch FETCH_SIZE $B
        pass s42_write WRITE_SIZE $B
        ;;
    pb)
        timeout -k 10 120 $R/zkevm-prover_amd/build/poseidon_bench > $O/poseidon_bench.txt 2>&1
        rc=$?; echo "[pmc_round] pb rc=$rc"; [ $rc -eq 0 ] || exit $rc
        ;;
    esac
done
cd $R
python3 tools/pmc_summary.py $O $TAG
