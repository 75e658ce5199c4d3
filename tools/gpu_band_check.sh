cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "band or sketch_sizes" > gpurun_out/gpu_band.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_band.log; exit 1; }
tail -3 gpurun_out/gpu_band.log
AP_N=2000 AP_S=10000 AP_PATH=band AP_L=5000000 timeout -k 10 300 python tools/ap_bench.py > gpurun_out/ap_band.json 2>&1 || { echo "ap band failed"; cat gpurun_out/ap_band.json; exit 1; }
cat gpurun_out/ap_band.json
AP_N=2000 AP_S=10000 AP_PATH=merge AP_L=5000000 AP_ITERS=1 timeout -k 10 300 python tools/ap_bench.py > gpurun_out/ap_merge.json 2>&1 || { echo "ap merge failed"; cat gpurun_out/ap_merge.json; exit 1; }
cat gpurun_out/ap_merge.json
