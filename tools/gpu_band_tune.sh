cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "band or sketch_sizes" > gpurun_out/gpu_band.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_band.log; exit 1; }
tail -2 gpurun_out/gpu_band.log
DREPHIP_BAND_GEOM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "band" > gpurun_out/gpu_band1.log 2>&1 || { echo "tests geom1 failed"; tail -40 gpurun_out/gpu_band1.log; exit 1; }
tail -2 gpurun_out/gpu_band1.log
for g in 0 1; do for cap in 384 512 768 1024; do
DREPHIP_BAND_GEOM=$g AP_N=2000 AP_S=10000 AP_PATH=band AP_CAP=$cap AP_L=5000000 AP_SAMPLE=20000 timeout -k 10 200 python tools/ap_bench.py 2>/dev/null > gpurun_out/ap_band_${g}_${cap}.json || { echo "ap band $g $cap failed"; exit 1; }
echo "geom $g cap $cap: $(cat gpurun_out/ap_band_${g}_${cap}.json)"
done; done
