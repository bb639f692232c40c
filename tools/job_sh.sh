cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_sharded_cpp.py -m gpu > gpurun_out/pt_sh.log 2>&1 || { tail -40 gpurun_out/pt_sh.log; exit 1; }
tail -3 gpurun_out/pt_sh.log
