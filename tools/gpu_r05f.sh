#!/bin/bash
# persistent NTT pass: parity of the NTT / LDE paths, then A/B of the LDE and the STARK
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_rb.py tests/test_gpu_large.py -k "ntt or lde or extend" > gpurun_out/r05f_tests.log 2>&1 || { tail -30 gpurun_out/r05f_tests.log; exit 1; }
tail -2 gpurun_out/r05f_tests.log
AB_DIRS="lib lib_w4 lib_ab" tools/ab_lib.sh lde --workload lde --steps 5 --warmup 2 || exit $?
AB_DIRS="lib lib_w4 lib_ab" tools/ab_lib.sh st --workload stark --steps 5 --warmup 2 --no-lde --no-handoff --no-s42 --no-sharded || exit $?
