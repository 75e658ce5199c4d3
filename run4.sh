cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; exit 1; }
