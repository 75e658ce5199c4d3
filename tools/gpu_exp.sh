cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "allpairs or dropin" > gpurun_out/gpu_ap.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_ap.log; exit 1; }
tail -2 gpurun_out/gpu_ap.log
for cfg in "1000 1000 table 0" "6000 1000 table 0" "1000 1000 table 1" "6000 1000 table 1" "2000 10000 band 0"; do
set -- $cfg
if [ $4 = 1 ]; then export DREPHIP_AP_ONEWG=1; else unset DREPHIP_AP_ONEWG; fi
AP_N=$1 AP_S=$2 AP_PATH=$3 AP_L=5000000 AP_SAMPLE=20000 timeout -k 10 200 python tools/ap_bench.py 2>gpurun_out/exp.err > gpurun_out/exp.json || { echo "ap $cfg failed"; cat gpurun_out/exp.err; exit 1; }
echo "$cfg: $(python3 -c "import json; d=json.load(open('gpurun_out/exp.json')); print(min(d['allpairs_ms']), d['pairs_per_s'], d['sample_pairs_exact'])")"
done
