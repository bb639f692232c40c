#!/bin/bash
# Per-dispatch counters of one north-star proof (fork-9 widths + the
# zkEVM-shaped programs, 2^23 rows, one GPU, lean plan): VALU / waves, HBM
# fetch and write in separate passes (MI355X_MICROARCH.md), each its own
# rocprofv3 run under its own time limit.  Summarise with
# tools/pmc_northstar_sum.py.  GPU box.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/nspmc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --workload stark --zkevm-shaped --log-n 23 --steps 1 --warmup 0 --no-cpu --no-lde --no-handoff --no-s42 --no-sharded"
for pass in "sq:SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
    name=${pass%%:*}
    ctr=${pass#*:}
    timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d $O/$name -o p --output-format csv -- $B > $O/$name.log 2>&1
    rc=$?
    echo "[pmc_northstar] $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
