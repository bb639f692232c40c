#!/bin/bash
# A/B of two builds of libzkgpu on one box, alternating (A B A B):
#   A = zkevm-prover_amd/lib, B = zkevm-prover_amd/lib_ab (ZKGPU_LIB_DIR)
# Usage (GPU box): tools/ab_lib.sh <label> <bench.py args...>
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
L=$1
shift
for r in 1 2; do
    for v in A B; do
        if [ $v = B ]; then export ZKGPU_LIB_DIR=$PWD/zkevm-prover_amd/lib_ab; else unset ZKGPU_LIB_DIR; fi
        timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab_${L}_$v$r.json 2> gpurun_out/ab_${L}_$v$r.err || exit $?
        echo "$L $v run $r: $(python -c "import json;d=json.loads(open('gpurun_out/ab_${L}_$v$r.json').read().strip().splitlines()[-1]);print(d['value'],d['unit'],(d.get('lde') or {}).get('value',''))")"
    done
done
unset ZKGPU_LIB_DIR
