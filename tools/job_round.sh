#!/bin/bash
# GPU test suite + the default bench line (what the driver runs at round end)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -c 600 $O/bench.log
