#!/bin/bash
# A/B: NTT kernels compiled with -amdgpu-sched-strategy=max-ilp (lib_ilp) vs default (lib)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ilp
mkdir -p $O
L2=$(pwd)/zkevm-prover_amd/lib_ilp
ZKGPU_LIB_DIR=$L2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "ntt or lde or extend" > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for rep in 1 2; do
for v in lib ilp; do
  for l3 in 0 1; do
    if [ $v = ilp ]; then export ZKGPU_LIB_DIR=$L2; else unset ZKGPU_LIB_DIR; fi
    ZKGPU_LDE3=$l3 timeout -k 10 200 python bench.py --workload lde --no-cpu --steps 10 --warmup 3 > $O/lde_${v}_${l3}_$rep.json 2> $O/lde_${v}_${l3}_$rep.err || exit $?
    python -c "import json; d=json.load(open('$O/lde_${v}_${l3}_$rep.json')); print('$v lde3=$l3 rep $rep', d['value'], d.get('ms_per_step'))"
  done
done
done
