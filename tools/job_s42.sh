cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload step42ns --s42-scale 0.25 --s42-jit --no-cpu --steps 3 --warmup 1 > gpurun_out/s42_w0.json 2> gpurun_out/s42_w0.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/s42_w0.json')); print('default', d['value'], d['unit'], d['ms_per_step'])"
ZKGPU_ZXP_JIT_WAVES=3 timeout -k 10 600 python bench.py --workload step42ns --s42-scale 0.25 --s42-jit --no-cpu --steps 3 --warmup 1 > gpurun_out/s42_w3.json 2> gpurun_out/s42_w3.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/s42_w3.json')); print('waves3', d['value'], d['unit'], d['ms_per_step'])"
