#!/bin/bash
# sharded / bench-rank tests after the host-exchange creation change, then A/B of the zkEVM-shaped proof
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_sharded_cpp.py tests/test_gpu_sharded_full.py tests/test_gpu_bench_ranks.py tests/test_gpu_batch_prover.py tests/test_gpu_zkevm_shaped.py > gpurun_out/r05k_tests.log 2>&1 || { tail -30 gpurun_out/r05k_tests.log; exit 1; }
tail -2 gpurun_out/r05k_tests.log
tools/ab_lib.sh zk --workload stark-sharded --zkevm-shaped --log-n 22 --steps 3 --warmup 1 || exit $?
