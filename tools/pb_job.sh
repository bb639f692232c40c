cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 build/poseidon_bench > gpurun_out/pb.txt 2>&1 || exit $?
timeout -k 10 120 build/instbench > gpurun_out/instbench.json 2> gpurun_out/instbench.err
