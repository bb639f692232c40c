#!/bin/bash
# LDS column cache A/B on the zkEVM-shaped quotient (ZKGPU_ZXP_JIT_LCACHE slots per lane; 0 = off),
# full-size parity first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lcache
mkdir -p $O
export ZKGPU_JIT_LOG=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_parser.py::test_step42ns_shaped_jit_gpu_equals_oracle" tests/test_gpu_parser.py::test_zkevm_shaped_programs_gpu_equal_oracle > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for rep in 1 2; do
for v in 12 0 8 16; do
  ZKGPU_ZXP_JIT_LCACHE=$v timeout -k 10 300 python bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 --warmup 1 > $O/l${v}_$rep.json 2> $O/l${v}_$rep.err || exit $?
  python -c "import json; d=[json.loads(l) for l in open('$O/l${v}_$rep.json') if l.startswith('{\"metric')][-1]; print('lcache $v rep $rep', d['value'], d['ms_per_step'])"
done
done
grep -h "cache miss" $O/*.err | head -5
