cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# issue / wait / memory-instruction counters of the quarter-size step42ns-shaped compiled kernel (current default)
B="python3 $GRAFT_REPO_ROOT/bench.py --workload step42ns --s42-scale 0.25 --s42-jit --no-cpu --steps 3 --warmup 1"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s42n_ic1 -o p --output-format csv -- $B > $GRAFT_REPO_ROOT/gpurun_out/s42n_ic1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s42n_ic2 -o p --output-format csv -- $B > $GRAFT_REPO_ROOT/gpurun_out/s42n_ic2.log 2>&1 || exit $?
echo done
