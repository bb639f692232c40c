cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# quarter-size step42ns-shaped compiled kernel at 2^24 rows: limb table (KAS) and column pointers (CPAS) read through
# FLAT (0) / global (1) / constant = scalar (4) loads
B="python3 $GRAFT_REPO_ROOT/bench.py --workload step42ns --s42-scale 0.25 --s42-jit --no-cpu --steps 3 --warmup 1"
for v in "1 0" "0 4" "1 4" "4 4"; do
  set -- $v
  ZKGPU_ZXP_JIT_KAS=$1 ZKGPU_ZXP_JIT_CPAS=$2 timeout -k 10 300 $B > gpurun_out/kas_$1$2.json 2> gpurun_out/kas_$1$2.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/kas_$1$2.json')); print('kas $1 cpas $2', d['value'], d['unit'], d['ms_per_step'])"
done
