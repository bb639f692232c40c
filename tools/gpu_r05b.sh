#!/bin/bash
# round-5 GPU check: the sharded prover (calculateH1H2 and FRI over the ranks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT tests/test_gpu_sharded_cpp.py tests/test_gpu_stark.py > gpurun_out/r05b_sharded.log 2>&1
rc=$?; tail -3 gpurun_out/r05b_sharded.log; exit $rc
