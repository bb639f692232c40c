#!/bin/bash
# round-5 check of the fused last tree levels (k_merkle_tail_lp), the batched
# calculateZ (zkgpu_calculate_z_many_dev) and the stage timers between stream
# marks (no synchronisation per stage): the Merkle / proof parity tests, then
# A/B (this tree's lib vs lib_ab) of the config-4 and zkEVM-shaped proofs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_stark.py tests/test_gpu_full_parity.py tests/test_gpu_bctree.py \
    tests/test_gpu_sharded_cpp.py tests/test_gpu_zkevm_shaped.py tests/test_gpu_batch_prover.py \
    > gpurun_out/r05o_tests.log 2>&1 || { tail -30 gpurun_out/r05o_tests.log; exit 1; }
tail -2 gpurun_out/r05o_tests.log
tools/ab_lib.sh c4 --workload stark --no-lde --no-handoff --no-s42 --no-sharded --steps 10 --warmup 2 || exit $?
tools/ab_lib.sh c4b --workload stark --no-lde --no-handoff --no-s42 --no-sharded --steps 10 --warmup 2 || exit $?
tools/ab_lib.sh zk --workload stark-sharded --zkevm-shaped --log-n 22 --steps 3 --warmup 1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/ab_c4_lib1.json').read().strip().splitlines()[-1]);print(json.dumps(d.get('stages_ms')))"
