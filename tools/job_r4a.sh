set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded_cpp.py tests/test_gpu_zkevm_shaped.py tests/test_gpu_stark.py > gpurun_out/r4a_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r4a_bench.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/r4a_bench.json'));print(d['value'],d['unit']);print(json.dumps(d.get('sharded_one_proof'))[:3000])"
