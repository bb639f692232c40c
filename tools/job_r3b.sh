#!/bin/bash
# round 3: the quotient with the reference's column locality -- parity + bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parser.py > $O/parser.log 2>&1 || { tail -30 $O/parser.log; exit 1; }
tail -3 $O/parser.log
timeout -k 10 400 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['quotient_zkevm_shaped'])[:900])"
