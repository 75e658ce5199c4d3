set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed $?" >> gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed $?"; exit 1; }
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/prof.log 2>&1 || { echo "prof failed $?"; exit 1; }
