#!/bin/bash
# LDE (configs[1]) kernel timings: parity on the 3-pass sizes, then rocprofv3 --kernel-trace --stats of the lde bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "extend" > gpurun_out/lde_par.log 2>&1
rc=$?
tail -3 gpurun_out/lde_par.log
[ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/gpurun_out/lprof" -o run --output-format csv -- python3 "$ROOTDIR/bench.py" --workload lde --no-cpu --steps 5 --warmup 1 "$@" > "$ROOTDIR/gpurun_out/lprof.json" 2>&1
rc=$?
cd "$ROOTDIR"
cut -d, -f1-4 gpurun_out/lprof/run_kernel_stats.csv | grep -E "k_lde|k_ntt"
exit $rc
