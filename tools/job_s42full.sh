cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# the full-size kernel must come from the in-tree cache (tools/jit_prebuild.py --full): a compile on the box takes minutes
timeout -k 10 120 python tools/jit_prebuild.py --check --full > gpurun_out/s42f_check.txt 2>&1 || exit $?
cat gpurun_out/s42f_check.txt
if grep -q "NOT cached" gpurun_out/s42f_check.txt; then echo "full-size kernel not cached"; exit 1; fi
timeout -k 10 300 python bench.py --workload step42ns --s42-scale 1.0 --s42-jit --no-cpu --steps 3 --warmup 1 > gpurun_out/s42f_jit.json 2> gpurun_out/s42f_jit.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/s42f_jit.json')); print('full jit', d['value'], d['unit'], d['ms_per_step'], d.get('roofline'))"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s42f_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload step42ns --s42-scale 1.0 --s42-jit --no-cpu --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/s42f_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/s42f_prof.err || exit $?
echo done
