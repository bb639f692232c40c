#!/bin/bash
# round-5 final numbers: per-dispatch traces of one config-4 and one
# zkEVM-shaped proof (tools/gpu_trace.sh), then two default bench runs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_trace.sh || exit $?
for r in 1 2; do
    timeout -k 10 600 python bench.py > gpurun_out/r05m_bench$r.json 2> gpurun_out/r05m_bench$r.err || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/r05m_bench$r.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['unit'], 'lde', d['lde']['value'], 'frac', d['roofline']['frac'])"
done
