set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
