#!/bin/bash
# step42ns-shaped program: parity of the compiled kernels (quarter, full-size
# segmented) and the full-size timing at 2^24 rows, per segment
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parser.py \
    > gpurun_out/seg_test.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload step42ns --s42-jit --s42-scale 1 --steps 3 --warmup 1 \
    > gpurun_out/seg_bench.log 2>&1
rc=$?
tail -5 gpurun_out/seg_test.log
exit $rc
