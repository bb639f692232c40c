#!/bin/bash
# FETCH_SIZE calibration for 8-byte-per-lane column reads (tools/fetch_calib.hip)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/calib
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 $R/zkevm-prover_amd/build/fetch_calib > $O/times.json 2> $O/times.err || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/$c -o p --output-format csv -- \
        $R/zkevm-prover_amd/build/fetch_calib > $O/$c.log 2>&1 || exit $?
done
echo done
