#!/bin/bash
# round-5 check of the batched query openings and the generator's occupancy
# memo: the -m gpu suite, then A/B (this tree's lib vs lib_ab) of the config-4
# proof and the zkEVM-shaped proof; each step under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu \
    > gpurun_out/r05l_tests.log 2>&1 || { tail -30 gpurun_out/r05l_tests.log; exit 1; }
tail -2 gpurun_out/r05l_tests.log
tools/ab_lib.sh c4 --workload stark --no-lde --no-handoff --no-s42 --no-sharded --steps 10 --warmup 2 || exit $?
tools/ab_lib.sh zk --workload stark-sharded --zkevm-shaped --log-n 22 --steps 3 --warmup 1 || exit $?
