#!/bin/bash
# round-5 GPU check: the new full-domain parity tests, the sharded prover and
# the FRI kernels (each step under its own time limit; stop at the first
# fault / timeout)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_gpu_parity.py -k fri > gpurun_out/r05a_fri.log 2>&1
rc=$?; tail -3 gpurun_out/r05a_fri.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $PYT tests/test_gpu_sharded_cpp.py > gpurun_out/r05a_sharded.log 2>&1
rc=$?; tail -3 gpurun_out/r05a_sharded.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $PYT tests/test_gpu_full_parity.py -k zkevm_shaped > gpurun_out/r05a_full.log 2>&1
rc=$?; tail -3 gpurun_out/r05a_full.log; exit $rc
