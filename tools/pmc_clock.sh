#!/bin/bash
# Effective shader clock per kernel: GRBM_GUI_ACTIVE (GPU-busy cycles) over the
# kernel's duration, for the permutation microbenchmark (whose s_memtime /
# s_memrealtime probe gives the clock independently), the Merkle bench and
# the LDE bench.  Usage (GPU box): tools/pmc_clock.sh
set -u
R=${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/clk_pb -o p --output-format csv -- $R/build/poseidon_bench > $R/gpurun_out/clk_pb.txt 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/clk_merkle -o p --output-format csv -- python3 $R/bench.py --workload merkle --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/clk_merkle.txt 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/clk_lde -o p --output-format csv -- python3 $R/bench.py --workload lde --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/clk_lde.txt 2>&1 || exit $?
echo done
