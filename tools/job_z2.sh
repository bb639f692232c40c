cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_stark.py tests/test_gpu_sharded_cpp.py -m gpu > gpurun_out/pt_z2.log 2>&1 || { tail -30 gpurun_out/pt_z2.log; exit 1; }
tail -1 gpurun_out/pt_z2.log
for i in 1 2; do
timeout -k 10 400 python bench.py --no-cpu --no-lde --no-handoff --steps 3 --warmup 1 > gpurun_out/bench_z2.json 2> gpurun_out/bench_z2.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_z2.json')); s=d['stages_ms']; print(d['value'], 'Z', s['STARK_STEP_3_CALCULATE_Z'], d['kernels'].get('k_z_ratio'), d['kernels'].get('k_z_apply'))"
done
