cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# config-4 STARK at 2^23: column pointers of the small (unsplit) expression kernels through scalar loads or the compiler's choice
for v in d 4; do
  if [ $v = 4 ]; then export ZKGPU_ZXP_JIT_CPAS=4; fi
  timeout -k 10 300 python3 bench.py --workload stark --no-cpu --no-handoff --steps 3 --warmup 1 > gpurun_out/cpas_$v.json 2> gpurun_out/cpas_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/cpas_$v.json')); print('cpas $v', d['value'], d['unit'], d['ms_per_step']); print({k: v for k, v in d.get('stages_ms', {}).items() if 'EXPS' in k})"
done
