#!/bin/bash
# LDE (configs[1]) PMC passes, one counter group per rocprofv3 run:
#   HBM traffic (FETCH_SIZE, WRITE_SIZE) and SQ issue / stall counters per kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in "FETCH_SIZE:lpmc_fetch" "WRITE_SIZE:lpmc_write" \
            "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE:lpmc_sq"; do
    ctr=${pass%%:*}
    out=${pass##*:}
    cd /tmp
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d "$ROOTDIR/gpurun_out/$out" -o run --output-format csv \
        -- python3 "$ROOTDIR/bench.py" --workload lde --no-cpu --steps 2 --warmup 1 "$@" > /dev/null 2> "$ROOTDIR/gpurun_out/$out.err"
    rc=$?
    cd "$ROOTDIR"
    echo "[lde_pmc] $out rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
