#!/bin/bash
# round-3 close: GPU suite, smoke, default bench, rocprof kernel stats of the default bench and of the fork-9 2^22 proof
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${FINAL_TAG:-final3}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 $R/bench.py --no-cpu --no-sharded --no-handoff --no-s42 > $O/prof.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/proff9 -o p --output-format csv -- python3 $R/bench.py --workload stark-sharded --fork9 --log-n 22 --steps 3 --warmup 1 --no-cpu > $O/proff9.log 2>&1 || exit $?
echo done
