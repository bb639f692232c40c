#!/bin/bash
# Per-dispatch kernel traces of one timed proof (after one warmup proof):
# config-4 at 2^23 (the headline) and the zkEVM-shaped instance at 2^22, for
# the host-gap analysis (tools/trace_gaps.py).  Each step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/trace_c4" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload stark --no-cpu --no-lde --no-handoff --no-s42 --no-sharded --steps 1 --warmup 1 \
    > "$R/gpurun_out/trace_c4_bench.json" 2> "$R/gpurun_out/trace_c4.err" || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace -d "$R/gpurun_out/trace_zk" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload stark-sharded --zkevm-shaped --log-n 22 --no-cpu --steps 1 --warmup 1 \
    > "$R/gpurun_out/trace_zk_bench.json" 2> "$R/gpurun_out/trace_zk.err" || exit $?
echo traces ok
