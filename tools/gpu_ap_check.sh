# all-pairs kernels: parity tests + timings (development check; not part of the product)
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "allpairs or dropin or smoke" > gpurun_out/gpu_ap.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_ap.log; exit 1; }
tail -2 gpurun_out/gpu_ap.log
for cfg in "1000 1000 table 0" "6000 1000 table 0" "2000 10000 band 0" "2000 10000 band 1"; do
set -- $cfg
DREPHIP_BAND_GEOM=$4 AP_N=$1 AP_S=$2 AP_PATH=$3 AP_L=5000000 AP_SAMPLE=20000 timeout -k 10 200 python tools/ap_bench.py 2>/dev/null > gpurun_out/ap_$1_$2_$3_$4.json || { echo "ap $cfg failed"; exit 1; }
echo "$cfg: $(cat gpurun_out/ap_$1_$2_$3_$4.json)"
done
