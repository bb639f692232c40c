cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# LDS limb chunks: -O1 (default) vs -O2 (LDS reads vectorised, 258 VGPRs)
B="python3 $GRAFT_REPO_ROOT/bench.py --workload step42ns --s42-scale 0.25 --s42-jit --no-cpu --steps 3 --warmup 1"
timeout -k 10 300 $B > gpurun_out/o1.json 2> gpurun_out/o1.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/o1.json')); print('O1', d['value'], d['unit'], d['ms_per_step'])"
ZKGPU_ZXP_JIT_OPT=2 timeout -k 10 300 $B > gpurun_out/o2.json 2> gpurun_out/o2.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/o2.json')); print('O2', d['value'], d['unit'], d['ms_per_step'])"
