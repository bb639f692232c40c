#!/bin/bash
# GPU job runner for gpurun: each GPU step has its own time limit; the job
# stops at the first fault / abort / segfault / timeout (exit >= 124 or
# signal), but continues past an ordinary test failure (exit 1).
# Usage: tools/gpu_job.sh <step>...   steps: tests smoke bench prof pmc large
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() {
    local rc=$1 what=$2
    echo "[gpu_job] $what exit=$rc" | tee -a gpurun_out/job.log
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "[gpu_job] stopping after $what (rc=$rc)" | tee -a gpurun_out/job.log
        exit "$rc"
    fi
}
for step in "$@"; do
    case "$step" in
    tests)
        timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider --deselect tests/test_gpu_large.py \
            > gpurun_out/pytest_gpu.log 2>&1
        ok_or_stop $? "pytest -m gpu"
        tail -5 gpurun_out/pytest_gpu.log
        ;;
    large)
        timeout -k 10 900 python -m pytest tests/test_gpu_large.py -x -q -p no:cacheprovider \
            > gpurun_out/pytest_gpu_large.log 2>&1
        ok_or_stop $? "pytest large"
        tail -5 gpurun_out/pytest_gpu_large.log
        ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
        ok_or_stop $? "smoke"
        tail -3 gpurun_out/smoke.log
        ;;
    bench)
        timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
        ok_or_stop $? "bench"
        cat gpurun_out/bench.json
        ;;
    sweep)
        for b in 1 2 4 10 100; do
            ZKGPU_LDE_BATCH_COLS=$b timeout -k 10 300 python bench.py --no-cpu > gpurun_out/sweep_b$b.json 2>> gpurun_out/sweep.err
            ok_or_stop $? "bench batch=$b"
            echo "batch=$b $(python -c "import json;d=json.load(open('gpurun_out/sweep_b$b.json'));print(d['ms_per_step'],'ms',d['value'],'Gelem/s',d['kernels'])")"
        done
        ;;
    merkle)
        timeout -k 10 600 python bench.py --workload merkle --steps 3 --warmup 1 > gpurun_out/bench_merkle.json 2> gpurun_out/bench_merkle.err
        ok_or_stop $? "bench merkle"
        cat gpurun_out/bench_merkle.json
        ;;
    stark)
        timeout -k 10 300 python bench.py --workload stark --log-n 16 --steps 2 --warmup 1 --no-cpu \
            > gpurun_out/bench_stark16.json 2> gpurun_out/bench_stark16.err
        ok_or_stop $? "bench stark 2^16"
        cat gpurun_out/bench_stark16.json
        timeout -k 10 900 python bench.py --workload stark --steps 3 --warmup 1 \
            > gpurun_out/bench_stark.json 2> gpurun_out/bench_stark.err
        ok_or_stop $? "bench stark"
        cat gpurun_out/bench_stark.json
        ;;
    commit)
        timeout -k 10 600 python bench.py --workload commit --steps 3 --warmup 1 \
            > gpurun_out/bench_commit.json 2> gpurun_out/bench_commit.err
        ok_or_stop $? "bench commit"
        cat gpurun_out/bench_commit.json
        ;;
    starkprof)
        cd /tmp
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_stark" -o run \
            --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload stark --no-cpu --steps 2 --warmup 1 \
            > "$GRAFT_REPO_ROOT/gpurun_out/prof_stark_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_stark.err"
        rc=$?
        cd "$GRAFT_REPO_ROOT"
        ok_or_stop $rc "rocprofv3 stark"
        ;;
    prof)
        cd /tmp
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
            --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu \
            > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err"
        rc=$?
        cd "$GRAFT_REPO_ROOT"
        ok_or_stop $rc "rocprofv3 kernel-trace"
        find gpurun_out/prof -name "*stats*" | head
        ;;
    pmc)
        cd /tmp
        timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch" -o run \
            --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 2 --warmup 1 \
            > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.err"
        rc=$?
        cd "$GRAFT_REPO_ROOT"
        ok_or_stop $rc "rocprofv3 pmc FETCH_SIZE"
        cd /tmp
        timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write" -o run \
            --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 2 --warmup 1 \
            > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc_write.err"
        rc=$?
        cd "$GRAFT_REPO_ROOT"
        ok_or_stop $rc "rocprofv3 pmc WRITE_SIZE"
        cd /tmp
        timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_sqb" -o run \
            --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 2 --warmup 1 \
            > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc_sqb.err"
        rc=$?
        cd "$GRAFT_REPO_ROOT"
        ok_or_stop $rc "rocprofv3 pmc SQ_INSTS_VALU"
        ;;
    starkpmc)
        # 2^23 STARK proof: HBM traffic (separate FETCH / WRITE passes) and VALU issue per kernel
        for pass in "FETCH_SIZE:pmc_sfetch" "WRITE_SIZE:pmc_swrite" \
                    "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE:pmc_ssq"; do
            ctr=${pass%%:*}
            out=${pass##*:}
            cd /tmp
            timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/$out" -o run \
                --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload stark --no-cpu --steps 1 --warmup 0 \
                > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/$out.err"
            rc=$?
            cd "$GRAFT_REPO_ROOT"
            ok_or_stop $rc "rocprofv3 stark pmc $out"
        done
        ;;
    zxpsweep)
        for r in 1 2 4; do
            ZKGPU_ZXP_ROWS=$r timeout -k 10 300 python bench.py --workload stark --steps 2 --warmup 1 --no-cpu \
                > gpurun_out/zxp_r$r.json 2>> gpurun_out/zxp_sweep.err
            ok_or_stop $? "stark zxp rows=$r"
            echo "rows=$r $(python -c "import json;d=json.load(open('gpurun_out/zxp_r$r.json'));print(d['ms_per_step'],'ms', d['kernels']['k_zxp_eval'])")"
        done
        ;;
    sharded)
        timeout -k 10 600 python -m pytest tests/test_sharded_stark.py -x -q -p no:cacheprovider -m gpu \
            > gpurun_out/pytest_sharded.log 2>&1
        ok_or_stop $? "pytest sharded stark gpu"
        tail -3 gpurun_out/pytest_sharded.log
        timeout -k 10 600 python bench.py --workload stark-sharded --steps 3 --warmup 1 --no-cpu \
            > gpurun_out/bench_stark_sharded.json 2> gpurun_out/bench_stark_sharded.err
        ok_or_stop $? "bench stark-sharded"
        cat gpurun_out/bench_stark_sharded.json
        ;;
    jitsweep)
        # KLDS OPT WAVES
        for cfg in "0 1 0" "1 1 0" "1 2 0" "1 2 4" "1 2 3" "0 2 0"; do
            set -- $cfg
            ZKGPU_ZXP_JIT_KLDS=$1 ZKGPU_ZXP_JIT_OPT=$2 ZKGPU_ZXP_JIT_WAVES=$3 timeout -k 10 300 python bench.py --workload stark --steps 2 --warmup 1 --no-cpu \
                > gpurun_out/jit_$1_$2_$3.json 2>> gpurun_out/jit_sweep.err
            ok_or_stop $? "stark jit klds=$1 opt=$2 waves=$3"
            echo "klds=$1 opt=$2 waves=$3 $(python -c "import json;d=json.load(open('gpurun_out/jit_$1_$2_$3.json'));s=d['stages_ms'];print(d['ms_per_step'],'ms q',s['STARK_STEP_4_CALCULATE_EXPS_2NS'],'f',s['STARK_STEP_5_CALCULATE_EXPS'],'s2',s['STARK_STEP_2_CALCULATE_EXPS'],'s3',s['STARK_STEP_3_CALCULATE_EXPS'])")"
        done
        ;;
    jitopt)
        for o in d 2 d 2; do
            if [ "$o" = d ]; then unset ZKGPU_ZXP_JIT_OPT; else export ZKGPU_ZXP_JIT_OPT=$o; fi
            timeout -k 10 300 python bench.py --workload stark --steps 2 --warmup 1 --no-cpu \
                > gpurun_out/jito_$o.json 2>> gpurun_out/jito.err
            ok_or_stop $? "stark jit opt=$o"
            echo "opt=$o $(python -c "import json;d=json.load(open('gpurun_out/jito_$o.json'));s=d['stages_ms'];print(d['ms_per_step'],'ms q',s['STARK_STEP_4_CALCULATE_EXPS_2NS'],'f',s['STARK_STEP_5_CALCULATE_EXPS'],'s2',s['STARK_STEP_2_CALCULATE_EXPS'],'s3',s['STARK_STEP_3_CALCULATE_EXPS'])")"
        done
        unset ZKGPU_ZXP_JIT_OPT
        ;;
    nttsplit)
        for v in 0 1 0 1; do
            ZKGPU_NTT_SPLIT=$v timeout -k 10 300 python bench.py --no-cpu > gpurun_out/ntt_split_$v.json 2>> gpurun_out/ntt_split.err
            ok_or_stop $? "bench ntt split=$v"
            echo "split=$v $(python -c "import json;d=json.load(open('gpurun_out/ntt_split_$v.json'));print(d['ms_per_step'],'ms',d['value'],'Gelem/s',d['kernels'])")"
        done
        ;;
    evsweep)
        for cfg in "1 1" "2 1" "4 1" "1 4" "2 2" "2 4" "4 2" "4 4"; do
            set -- $cfg
            ZKGPU_EVMAP_G=$1 ZKGPU_EVMAP_U=$2 timeout -k 10 300 python bench.py --workload stark --steps 2 --warmup 1 --no-cpu \
                > gpurun_out/ev_$1_$2.json 2>> gpurun_out/ev_sweep.err
            ok_or_stop $? "stark evmap G=$1 U=$2"
            echo "G=$1 U=$2 $(python -c "import json;d=json.load(open('gpurun_out/ev_$1_$2.json'));print(d['ms_per_step'],'ms evmap',d['kernels']['k_evmap'])")"
        done
        ;;
    sqpmc)
        # VALU/SALU/SMEM issue and wave-state counters for every kernel of a 2^20 STARK proof
        cd /tmp
        timeout -s KILL 120 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/rocprof_counters.txt" 2>&1
        timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
            -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_sq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" \
            --workload stark --log-n 20 --no-cpu --steps 1 --warmup 0 > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc_sq.err"
        rc=$?
        cd "$GRAFT_REPO_ROOT"
        ok_or_stop $rc "rocprofv3 pmc SQ"
        ;;
    *)
        echo "unknown step $step"
        ;;
    esac
done
echo "[gpu_job] done" | tee -a gpurun_out/job.log
