#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT tests/test_gpu_batch_prover.py tests/test_gpu_sharded_cpp.py > gpurun_out/r05e_sharded.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_sharded.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 $PYT tests/test_gpu_full_parity.py > gpurun_out/r05e_full.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_full.log; exit $rc
