cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 1 0 1 0; do
  ZKGPU_NTT_HALF=$v timeout -k 10 300 python bench.py --workload lde --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_h$v.json 2> gpurun_out/ab.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab_h$v.json')); print('half=$v LDE', d['value'])"
done
