#!/bin/bash
# per-dispatch kernel trace of the zkEVM-shaped proof at 2^22 (one rank): GPU idle gaps inside a proof
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_zk -o run --output-format csv -- \
    python3 $R/bench.py --workload stark-sharded --zkevm-shaped --log-n 22 --steps 2 --warmup 1 --no-cpu \
    > $R/gpurun_out/trace_zk_bench.json 2> $R/gpurun_out/trace_zk.err
echo "rc=$?"
