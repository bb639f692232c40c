cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu --deselect tests/test_gpu_large.py --deselect tests/test_gpu_config4.py > gpurun_out/pt_w.log 2>&1 || { tail -40 gpurun_out/pt_w.log; exit 1; }
tail -2 gpurun_out/pt_w.log
for v in 1 0; do
ZKGPU_ZXP_JIT_AUTOWAVES=$v timeout -k 10 400 python bench.py --no-cpu --no-lde --no-handoff --steps 3 --warmup 1 > gpurun_out/bench_w$v.json 2> gpurun_out/bench_w.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_w$v.json')); s=d['stages_ms']; print('autowaves=$v', d['value'], 'q', s['STARK_STEP_4_CALCULATE_EXPS_2NS'], 'fri', s['STARK_STEP_5_CALCULATE_EXPS'], 'st2', s['STARK_STEP_2_CALCULATE_EXPS'], 'st3', s['STARK_STEP_3_CALCULATE_EXPS'])"
done
