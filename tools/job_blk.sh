cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# quarter-size step42ns-shaped compiled kernel at 2^24 rows (global limbs, scalar column pointers): source bytes per code block
B="python3 $GRAFT_REPO_ROOT/bench.py --workload step42ns --s42-scale 0.25 --s42-jit --no-cpu --steps 3 --warmup 1"
for v in 1024 1536 2048; do
  ZKGPU_ZXP_JIT_BLOCK=$v timeout -k 10 300 $B > gpurun_out/blk_$v.json 2> gpurun_out/blk_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/blk_$v.json')); print('block $v', d['value'], d['unit'], d['ms_per_step'])"
done
