cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_h1h2.py tests/test_gpu_stark.py -m gpu > gpurun_out/pt_h12.log 2>&1 || { tail -30 gpurun_out/pt_h12.log; exit 1; }
tail -3 gpurun_out/pt_h12.log
timeout -k 10 400 python bench.py --no-cpu --no-lde > gpurun_out/bench_h12.json 2> gpurun_out/bench_h12.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_h12.json')); print(d['value'], {k:v for k,v in d['stages_ms'].items() if 'H1H2' in k or 'TOTAL' in k})"
