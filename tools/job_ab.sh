cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_stark.py tests/test_gpu_sharded_cpp.py -m gpu > gpurun_out/pt_ab.log 2>&1 || { tail -30 gpurun_out/pt_ab.log; exit 1; }
tail -1 gpurun_out/pt_ab.log
for v in 0 1 0 1; do
  ZKGPU_LEAVES_W6=$v timeout -k 10 300 python bench.py --workload merkle --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_l$v.json 2> gpurun_out/ab.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab_l$v.json')); print('w6=$v merkle', d['value'], d['unit'])"
done
