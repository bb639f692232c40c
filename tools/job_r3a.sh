#!/bin/bash
# round 3: LDE column-batch A/B on the default bench, the row-sharded prover at W=1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3a
O=gpurun_out/r3a
timeout -k 10 300 python bench.py --no-cpu --no-s42 > $O/bench_b32.json 2> $O/bench_b32.err || exit $?
tail -c 300 $O/bench_b32.json; echo
ZKGPU_LDE_BATCH_COLS=100 timeout -k 10 300 python bench.py --no-cpu --no-s42 > $O/bench_b100.json 2> $O/bench_b100.err || exit $?
tail -c 300 $O/bench_b100.json; echo
timeout -k 10 300 python bench.py --workload stark-sharded --steps 3 --warmup 1 > $O/sharded_c4.json 2> $O/sharded_c4.err || exit $?
tail -c 300 $O/sharded_c4.json; echo
timeout -k 10 400 python bench.py --workload stark-sharded --fork9 --log-n 20 --steps 3 --warmup 1 > $O/sharded_f9.json 2> $O/sharded_f9.err || exit $?
tail -c 300 $O/sharded_f9.json; echo
