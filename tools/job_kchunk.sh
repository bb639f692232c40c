cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# LDS limb chunks (ZKGPU_ZXP_JIT_KCHUNK=1) on the quarter-size step42ns-shaped program: parity vs the oracle, then 2^24-row timing
ZKGPU_ZXP_JIT_KCHUNK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parser.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k jit > gpurun_out/kchunk_test.log 2>&1 || { tail -30 gpurun_out/kchunk_test.log; exit 1; }
tail -2 gpurun_out/kchunk_test.log
B="python3 $GRAFT_REPO_ROOT/bench.py --workload step42ns --s42-scale 0.25 --s42-jit --no-cpu --steps 3 --warmup 1"
for v in 0 1; do
  ZKGPU_ZXP_JIT_KCHUNK=$v timeout -k 10 300 $B > gpurun_out/kchunk_$v.json 2> gpurun_out/kchunk_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/kchunk_$v.json')); print('kchunk $v', d['value'], d['unit'], d['ms_per_step'])"
done
