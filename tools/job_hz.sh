cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_stark.py tests/test_gpu_bctree.py -m gpu > gpurun_out/pt_hz.log 2>&1 || { tail -40 gpurun_out/pt_hz.log; exit 1; }
tail -1 gpurun_out/pt_hz.log
for i in 1 2; do
timeout -k 10 300 python bench.py --workload lde --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_hz.json 2> gpurun_out/bench_hz.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_hz.json')); print('LDE', d['value'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['lde']['kernels'].items()} if 'lde' in d else d.get('kernels'))"
done
