#!/bin/bash
# (1) radix-256 pass with rare-branch butterflies vs select form (ablib/): LDE 6-pass / 3-pass, STARK
# (2) expression kernels with ZK_RB (ZKGPU_ZXP_JIT_RB=1) vs without: zkEVM-shaped quotient, parity first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rb2
mkdir -p $O
export ZKGPU_JIT_LOG=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_large.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
ZKGPU_ZXP_JIT_RB=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_parser.py::test_step42ns_shaped_jit_gpu_equals_oracle" tests/test_gpu_parser.py::test_zkevm_shaped_programs_gpu_equal_oracle > $O/parity_jit.log 2>&1 || { tail -30 $O/parity_jit.log; exit 1; }
tail -1 $O/parity_jit.log
for rep in 1 2; do
for v in rb base; do
  if [ $v = base ]; then export ZKGPU_LIB_DIR=$PWD/ablib; else unset ZKGPU_LIB_DIR; fi
  timeout -k 10 200 python bench.py --workload lde --no-cpu --steps 10 --warmup 3 > $O/lde_$v$rep.json 2> $O/lde_$v$rep.err || exit $?
  ZKGPU_LDE3=1 timeout -k 10 200 python bench.py --workload lde --no-cpu --steps 10 --warmup 3 > $O/lde3_$v$rep.json 2> $O/lde3_$v$rep.err || exit $?
  python -c "
import json
def last(f): return [json.loads(l) for l in open(f) if l.startswith('{\"metric')][-1]
a=last('$O/lde_$v$rep.json'); b=last('$O/lde3_$v$rep.json')
print('$v rep $rep', 'lde', a['value'], 'lde3', b['value'])"
done
unset ZKGPU_LIB_DIR
for j in 0 1; do
  ZKGPU_ZXP_JIT_RB=$j timeout -k 10 300 python bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 --warmup 1 > $O/q${j}_$rep.json 2> $O/q${j}_$rep.err || exit $?
  python -c "import json; d=[json.loads(l) for l in open('$O/q${j}_$rep.json') if l.startswith('{\"metric')][-1]; print('jit rb $j rep $rep', d['value'], d['ms_per_step'])"
done
done
grep -h "cache miss" $O/*.err | head -5
