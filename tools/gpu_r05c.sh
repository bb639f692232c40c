#!/bin/bash
# round-5 GPU check: the whole -m gpu suite (the large tests included), then
# smoke; each step under its own limit, stop at the first fault / timeout
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 1000 $PYT tests -m gpu > gpurun_out/r05c_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r05c_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05c_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_smoke.log; exit $rc
