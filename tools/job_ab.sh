cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 0 1 0 1; do
  ZKGPU_LEAVES_W6=$v timeout -k 10 300 python bench.py --workload merkle --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_l$v.json 2> gpurun_out/ab.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab_l$v.json')); print('w6=$v merkle', d['value'], d['unit'])"
done
