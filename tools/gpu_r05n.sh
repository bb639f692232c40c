#!/bin/bash
# round-5 check of the host compiler changes (Karatsuba scaling, Bloom column
# hazards, interned column memo): the expression-program GPU tests, then A/B
# (this tree's lib vs lib_ab) of the zkEVM-shaped and config-4 proofs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parser.py tests/test_gpu_zkevm_shaped.py tests/test_gpu_stark.py tests/test_gpu_full_parity.py \
    tests/test_gpu_batch_prover.py > gpurun_out/r05n_tests.log 2>&1 || { tail -30 gpurun_out/r05n_tests.log; exit 1; }
tail -2 gpurun_out/r05n_tests.log
tools/ab_lib.sh zk --workload stark-sharded --zkevm-shaped --log-n 22 --steps 3 --warmup 1 || exit $?
tools/ab_lib.sh c4 --workload stark --no-lde --no-handoff --no-s42 --no-sharded --steps 10 --warmup 2 || exit $?
