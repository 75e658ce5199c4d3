cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for cfg in "1000 1000 band 1024" "1000 1000 band 256" "2000 10000 band 1024"; do
set -- $cfg
DREPHIP_BAND_PROF=1 AP_ITERS=1 AP_N=$1 AP_S=$2 AP_PATH=$3 AP_CAP=$4 AP_L=5000000 AP_SAMPLE=2000 timeout -k 10 200 python tools/ap_bench.py 2>gpurun_out/exp.err > gpurun_out/exp.json || { echo "ap $cfg failed"; cat gpurun_out/exp.err; exit 1; }
echo "$cfg: $(python3 -c "import json; d=json.load(open('gpurun_out/exp.json')); print(min(d['allpairs_ms']), d['sample_pairs_exact'])") $(grep band gpurun_out/exp.err)"
done
