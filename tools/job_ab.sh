cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 0 3 4; do
  if [ $v = 0 ]; then unset ZKGPU_ZXP_JIT_WAVES; else export ZKGPU_ZXP_JIT_WAVES=$v; fi
  timeout -k 10 400 python bench.py --no-cpu --no-lde --no-handoff --steps 3 --warmup 1 > gpurun_out/ab_w$v.json 2> gpurun_out/ab_w$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab_w$v.json')); s=d['stages_ms']; print('waves=$v', d['value'], 'q', s['STARK_STEP_4_CALCULATE_EXPS_2NS'], 'fri', s['STARK_STEP_5_CALCULATE_EXPS'], 'st2', s['STARK_STEP_2_CALCULATE_EXPS'])"
done
