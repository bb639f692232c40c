#!/bin/bash
# LDS column cache x rows per thread on the zkEVM-shaped quotient; parity first (default form)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lcache2
mkdir -p $O
export ZKGPU_JIT_LOG=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_parser.py::test_step42ns_shaped_jit_gpu_equals_oracle" tests/test_gpu_parser.py::test_zkevm_shaped_programs_gpu_equal_oracle > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
ZKGPU_ZXP_JIT_ROWS=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_parser.py::test_step42ns_shaped_jit_gpu_equals_oracle" > $O/parity_r2.log 2>&1 || { tail -30 $O/parity_r2.log; exit 1; }
tail -1 $O/parity_r2.log
for rep in 1 2; do
for v in "1 12" "2 12" "1 16"; do
  set -- $v
  ZKGPU_ZXP_JIT_ROWS=$1 ZKGPU_ZXP_JIT_LCACHE=$2 timeout -k 10 300 python bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 --warmup 1 > $O/r$1_$2_$rep.json 2> $O/r$1_$2_$rep.err || exit $?
  python -c "import json; d=[json.loads(l) for l in open('$O/r$1_$2_$rep.json') if l.startswith('{\"metric')][-1]; print('rows $1 lcache $2 rep $rep', d['value'], d['ms_per_step'])"
done
done
grep -h "cache miss" $O/*.err | head -5
