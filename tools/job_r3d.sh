#!/bin/bash
# round 3: driver tests (fork-9 widths over 8 ranks) + the default bench with the one-proof child runs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_sharded_cpp.py tests/test_gpu_batch_prover.py > $O/bp.log 2>&1
rc=$?
grep -E "FAIL|passed|failed" $O/bp.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d.get('sharded_one_proof'))[:1500])"
