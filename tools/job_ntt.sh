cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_stark.py tests/test_gpu_bctree.py -m gpu > gpurun_out/pt_ntt.log 2>&1 || { tail -40 gpurun_out/pt_ntt.log; exit 1; }
tail -3 gpurun_out/pt_ntt.log
timeout -k 10 400 python bench.py --workload lde --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_lde.json 2> gpurun_out/bench_lde.err || exit $?
timeout -k 10 400 python bench.py --no-cpu --no-handoff --steps 3 --warmup 1 > gpurun_out/bench_ntt.json 2> gpurun_out/bench_ntt.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_lde.json')); print('LDE', d['value'], d['roofline']['frac']); d=json.load(open('gpurun_out/bench_ntt.json')); print('STARK', d['value'], d['lde']['value'])"
