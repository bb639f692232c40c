#!/bin/bash
# fork-9 widths on one GPU at 2^22 (the row-sharded prover at one rank) + JIT cache-miss log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/f9
mkdir -p $O
export ZKGPU_JIT_LOG=1
timeout -k 10 400 python -u bench.py --workload stark-sharded --fork9 --log-n 22 --steps 3 --warmup 1 --no-cpu > $O/f9_22.json 2> $O/f9_22.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-handoff --steps 3 --warmup 1 > $O/c4.json 2> $O/c4.err || exit $?
grep -h "cache miss" $O/*.err | head -20
python - <<'PY'
import json
d = json.load(open("gpurun_out/f9/f9_22.json"))
print(d["value"], d["ms_per_step"], json.dumps(d.get("stages_ms")))
d = json.load(open("gpurun_out/f9/c4.json"))
print("config4", d["value"])
PY
