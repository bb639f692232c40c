set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_IFETCH SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmc_ic1 -o p -- python3 $R/bench.py --workload merkle --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/pmc_ic1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $R/gpurun_out/pmc_ic2 -o p -- python3 $R/bench.py --workload merkle --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/pmc_ic2.log 2>&1
echo done
