#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_h1h2.py -m gpu > gpurun_out/r05d_h1h2.log 2>&1
rc=$?; tail -3 gpurun_out/r05d_h1h2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 $PYT tests/test_gpu_batch_prover.py tests/test_gpu_sharded_cpp.py > gpurun_out/r05d_sharded.log 2>&1
rc=$?; tail -3 gpurun_out/r05d_sharded.log; exit $rc
