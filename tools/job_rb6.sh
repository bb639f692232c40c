#!/bin/bash
# expression kernels with ZK_RB (add / sub / reduction rare corrections behind uniform branches) vs without:
# parity, zkEVM-shaped quotient, config-4 STARK expression stages
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rb6
mkdir -p $O
export ZKGPU_JIT_LOG=1
ZKGPU_ZXP_JIT_RB=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_parser.py::test_step42ns_shaped_jit_gpu_equals_oracle" tests/test_gpu_parser.py::test_zkevm_shaped_programs_gpu_equal_oracle \
  tests/test_gpu_stark.py::test_full_proof_bit_exact_jit tests/test_gpu_stark.py::test_fork9_widths_proof_bit_exact_jit > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for rep in 1 2; do
for j in 0 1; do
  ZKGPU_ZXP_JIT_RB=$j timeout -k 10 300 python bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 --warmup 1 > $O/q${j}_$rep.json 2> $O/q${j}_$rep.err || exit $?
  ZKGPU_ZXP_JIT_RB=$j timeout -k 10 300 python bench.py --no-cpu --no-sharded --no-handoff --no-s42 --no-lde --steps 5 --warmup 2 > $O/s${j}_$rep.json 2> $O/s${j}_$rep.err || exit $?
  python -c "
import json
def last(f): return [json.loads(l) for l in open(f) if l.startswith('{\"metric')][-1]
q=last('$O/q${j}_$rep.json'); s=last('$O/s${j}_$rep.json'); st=s['stages_ms']
print('jit rb $j rep $rep', 'quotient', q['value'], 'stark', s['value'], 'exps', st['STARK_STEP_4_CALCULATE_EXPS_2NS'], st['STARK_STEP_5_CALCULATE_EXPS'])"
done
done
grep -h "cache miss" $O/*.err | head -5
