#!/bin/bash
# round-5 final: the whole -m gpu suite, smoke, then three default bench runs
# (profiles/r05_final_bench.json); each step under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu \
    > gpurun_out/r05z_gpu.log 2>&1 || { tail -30 gpurun_out/r05z_gpu.log; exit 1; }
tail -1 gpurun_out/r05z_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z_smoke.log 2>&1 || { tail -5 gpurun_out/r05z_smoke.log; exit 1; }
tail -1 gpurun_out/r05z_smoke.log
for r in 1 2 3; do
    timeout -k 10 400 python bench.py > gpurun_out/r05z_bench$r.json 2> gpurun_out/r05z_bench$r.err || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/r05z_bench$r.json').read().strip().splitlines()[-1]);print('bench', d['value'], 'lde', d['lde']['value'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])"
done
