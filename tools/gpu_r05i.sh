#!/bin/bash
# host preparation of the compiled expression kernels: parity, then A/B (zkEVM-shaped 2^22, config-4 2^23)
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zkevm_shaped.py tests/test_gpu_parser.py tests/test_gpu_full_parity.py tests/test_gpu_stark.py tests/test_gpu_sharded_cpp.py > gpurun_out/r05i_tests.log 2>&1 || { tail -30 gpurun_out/r05i_tests.log; exit 1; }
tail -2 gpurun_out/r05i_tests.log
tools/ab_lib.sh zk --workload stark-sharded --zkevm-shaped --log-n 22 --steps 3 --warmup 1 || exit $?
tools/ab_lib.sh c4 --workload stark --steps 5 --warmup 2 --no-lde --no-handoff --no-s42 --no-sharded || exit $?
