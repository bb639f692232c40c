cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# quarter-size step42ns-shaped compiled kernel at 2^24 rows: workgroup barrier every n code blocks (ZKGPU_ZXP_JIT_SYNC) A/B,
# then the instruction-fetch counters of the default kernel
B="python3 $GRAFT_REPO_ROOT/bench.py --workload step42ns --s42-scale 0.25 --s42-jit --no-cpu --steps 3 --warmup 1"
for v in 0 1 4; do
  ZKGPU_ZXP_JIT_SYNC=$v timeout -k 10 300 $B > gpurun_out/s42s_$v.json 2> gpurun_out/s42s_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/s42s_$v.json')); print('sync $v', d['value'], d['unit'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_IFETCH SQ_ACTIVE_INST_ANY --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s42_ic1 -o p --output-format csv -- $B > $GRAFT_REPO_ROOT/gpurun_out/s42_ic1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s42_ic2 -o p --output-format csv -- $B > $GRAFT_REPO_ROOT/gpurun_out/s42_ic2.log 2>&1 || exit $?
echo done
