#!/bin/bash
# zkEVM-sized (full) step42ns-shaped quotient at 2^24 rows, default segments:
# parity (2^16, vs oracle), kernel-trace stats, and counter passes
# (issue / wait classes, instruction mix, HBM fetch and write bytes)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s42pmc
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_parser.py > $O/test.log 2>&1 || exit $?
B="python3 $R/bench.py --workload step42ns --s42-scale 1 --s42-jit --no-cpu --steps 3 --warmup 1"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/stats -o p --output-format csv -- $B > $O/stats.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -d $O/p1 -o p --output-format csv -- $B > $O/p1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_IFETCH SQ_ACTIVE_INST_SCA --kernel-trace -d $O/p2 -o p --output-format csv -- $B > $O/p2.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/p3 -o p --output-format csv -- $B > $O/p3.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/p4 -o p --output-format csv -- $B > $O/p4.log 2>&1 || exit $?
echo done
