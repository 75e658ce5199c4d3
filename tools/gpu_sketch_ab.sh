# sketch kernel A/B (development): parity tests under each variant + bench
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for v in ${SK_VARIANTS:-5 4}; do
DREPHIP_SKETCH_KERNEL=$v timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "${SK_TESTS:-sketch or synth or dropin or reference}" > gpurun_out/gpu_sk$v.log 2>&1 || { echo "tests v$v failed"; tail -30 gpurun_out/gpu_sk$v.log; exit 1; }
tail -1 gpurun_out/gpu_sk$v.log
DREPHIP_SKETCH_KERNEL=$v timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_sk$v.json 2>/dev/null || { echo "bench v$v failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_sk$v.json')); print('v$v', d['ms_per_step'], d['kernels_rank0']['sketch_hash_ms_avg'])"
done
