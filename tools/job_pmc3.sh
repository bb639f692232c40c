#!/bin/bash
# round-3 close: per-kernel VALU / HBM counters of one 2^23 proof (tools/stark_pmc.py) and effective clocks
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
tools/gpu_job.sh starkpmc > gpurun_out/starkpmc.log 2>&1 || { tail -20 gpurun_out/starkpmc.log; exit 1; }
python3 tools/stark_pmc.py gpurun_out gpurun_out/r03_stark_pmc.json > gpurun_out/stark_pmc_summary.txt || exit $?
head -8 gpurun_out/stark_pmc_summary.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/clk_merkle -o p --output-format csv -- python3 $R/bench.py --workload merkle --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/clk_merkle.txt 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/clk_lde -o p --output-format csv -- python3 $R/bench.py --workload lde --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/clk_lde.txt 2>&1 || exit $?
cd $R && python3 tools/clock_summary.py gpurun_out/r03_clock.json gpurun_out/clk_merkle gpurun_out/clk_lde
