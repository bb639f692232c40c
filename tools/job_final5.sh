#!/bin/bash
# round-3 close: isolated permutation benchmark (current poseidon_perm.hpp) and the default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out/final5
timeout -k 10 120 zkevm-prover_amd/build/poseidon_bench > gpurun_out/final5/r03_poseidon_bench.txt 2>&1 || exit $?
cat gpurun_out/final5/r03_poseidon_bench.txt | tail -8
cp gpurun_out/final5/r03_poseidon_bench.txt profiles/r03_poseidon_bench.txt
timeout -k 10 300 python -u bench.py > gpurun_out/final5/bench.json 2> gpurun_out/final5/bench.err || exit $?
echo done
