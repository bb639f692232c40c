#!/bin/bash
# A/B of builds of libzkgpu on one box, alternating (A B A B ...):
#   AB_DIRS (default "lib lib_ab"): directories under zkevm-prover_amd/ holding
#   a build of both libraries (ZKGPU_LIB_DIR); the first is the tree's own lib
# Usage (GPU box): [AB_DIRS="lib lib_ab lib_c"] tools/ab_lib.sh <label> <bench.py args...>
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
L=$1
shift
DIRS=${AB_DIRS:-lib lib_ab}
for r in 1 2; do
    for v in $DIRS; do
        export ZKGPU_LIB_DIR=$PWD/zkevm-prover_amd/$v
        timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab_${L}_$v$r.json 2> gpurun_out/ab_${L}_$v$r.err || exit $?
        echo "$L $v run $r: $(python -c "import json;d=json.loads(open('gpurun_out/ab_${L}_$v$r.json').read().strip().splitlines()[-1]);print(d['value'],d['unit'],(d.get('lde') or {}).get('value',''))")"
    done
done
unset ZKGPU_LIB_DIR
