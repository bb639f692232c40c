#!/bin/bash
# round 3 profiles: kernel-trace stats of the default STARK bench (replica leg
# only) and the LDE PMC passes (HBM bytes + SQ counters)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
O=$ROOTDIR/gpurun_out/r3prof
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats -o p --output-format csv -- python3 $ROOTDIR/bench.py --no-cpu --no-s42 --no-sharded --no-handoff > $O/stats_bench.json 2> $O/stats.err || exit $?
cd $ROOTDIR
tools/lde_pmc.sh || exit $?
mv gpurun_out/lpmc_* $O/ 2>/dev/null
echo done
