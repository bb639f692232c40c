#!/bin/bash
# Where the NTT pass kernels' wave time goes (bench.py --workload lde):
# SQ_WAIT_ANY (waitcnt: memory / LDS), SQ_WAIT_INST_ANY (ready, not issued),
# SQ_ACTIVE_INST_* by class, LDS bank conflicts.  Two passes (SQ counter limit).
set -u
R=${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -d $R/gpurun_out/ntt_st1 -o p --output-format csv -- python3 $R/bench.py --workload lde --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/ntt_st1.txt 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA --kernel-trace -d $R/gpurun_out/ntt_st2 -o p --output-format csv -- python3 $R/bench.py --workload lde --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/ntt_st2.txt 2>&1 || exit $?
echo done
