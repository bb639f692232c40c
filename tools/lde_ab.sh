cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for x in 0 1; do
  ZKGPU_LDE3_XCD=$x timeout -k 10 120 python bench.py --workload lde --no-cpu --steps 10 --warmup 2 > gpurun_out/ab_xcd$x.json 2>/dev/null || exit 1
  echo "xcd=$x $(grep -o '"value": [0-9.]*' gpurun_out/ab_xcd$x.json | head -1)"
done
ZKGPU_LDE3=0 timeout -k 10 120 python bench.py --workload lde --no-cpu --steps 10 --warmup 2 > gpurun_out/ab_old.json 2>/dev/null || exit 1
echo "old $(grep -o '"value": [0-9.]*' gpurun_out/ab_old.json | head -1)"
