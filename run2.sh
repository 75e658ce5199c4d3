cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 120 ./tools/valu_microbench > gpurun_out/microbench.json 2> gpurun_out/microbench.err
