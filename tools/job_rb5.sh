#!/bin/bash
# rare-branch MDS and dot-product reductions in Poseidon (lib/) vs S-box only (ablib/): parity, LDE, Merkle, STARK
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rb5
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_stark.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for rep in 1 2; do
for v in fin base; do
  if [ $v = base ]; then export ZKGPU_LIB_DIR=$PWD/ablib; else unset ZKGPU_LIB_DIR; fi
  timeout -k 10 200 python bench.py --workload lde --no-cpu --steps 10 --warmup 3 > $O/lde_$v$rep.json 2> $O/lde_$v$rep.err || exit $?
  timeout -k 10 200 python bench.py --workload merkle --no-cpu --steps 5 --warmup 2 > $O/mk_$v$rep.json 2> $O/mk_$v$rep.err || exit $?
  timeout -k 10 300 python bench.py --no-cpu --no-sharded --no-handoff --no-s42 --no-lde --steps 5 --warmup 2 > $O/stark_$v$rep.json 2> $O/stark_$v$rep.err || exit $?
  python -c "
import json
def last(f): return [json.loads(l) for l in open(f) if l.startswith('{\"metric')][-1]
a=last('$O/lde_$v$rep.json'); m=last('$O/mk_$v$rep.json'); c=last('$O/stark_$v$rep.json')
print('$v rep $rep', 'lde', a['value'], 'merkle', m['value'], 'stark', c['value'], 'step1 LDE', c['stages_ms']['STARK_STEP_1_LDE'], 'step1 tree', c['stages_ms']['STARK_STEP_1_MERKLETREE'])"
done
done
