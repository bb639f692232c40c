set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_sharded_cpp.py tests/test_gpu_lean.py tests/test_gpu_bench_ranks.py > gpurun_out/r06b_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r06b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload stark --zkevm-shaped --log-n 23 --steps 3 --warmup 1 --no-cpu --no-lde --no-handoff --no-s42 --no-sharded > gpurun_out/r06b_ns.json 2> gpurun_out/r06b_ns.err
rc=$?; tail -c 3000 gpurun_out/r06b_ns.json; exit $rc
