#!/bin/bash
# after the xDivXSub kernel specialisation: stark + sharded tests, default bench, kernel stats
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/final3b
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_stark.py tests/test_gpu_sharded_cpp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 $R/bench.py --no-cpu --no-sharded --no-handoff --no-s42 > $O/prof.log 2>&1 || exit $?
echo done
