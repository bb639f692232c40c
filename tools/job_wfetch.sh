#!/bin/bash
# quotient HBM fetch bytes at 4 vs 2 waves per SIMD (rows in flight vs L2 reuse)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
O=$ROOTDIR/gpurun_out/wfetch
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for w in 4 2; do
  ZKGPU_ZXP_SEG_WAVES=$w timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/w$w -o p --output-format csv -- python3 $ROOTDIR/bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 2 --warmup 1 > $O/w$w.json 2> $O/w$w.err || exit $?
done
echo done
