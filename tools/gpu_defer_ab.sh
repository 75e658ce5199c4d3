cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_t4.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_t4.log; exit 1; }
tail -2 gpurun_out/gpu_t4.log
for d in 0 1; do
  SHARD_TIMING=0 SHARD_DEFER=$d timeout -k 10 120 python tools/shard_step.py 1000 8 0 30 > gpurun_out/shard_d$d.json 2>/dev/null || { echo "shard $d failed"; exit 1; }
  cat gpurun_out/shard_d$d.json
done
for d in 0 1 0 1; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --defer-check $d --steps 10 > gpurun_out/bench_d$d.json 2> gpurun_out/bench_d$d.err || { echo "bench $d failed"; tail gpurun_out/bench_d$d.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_d$d.json')); print('defer', $d, d['ms_per_step'], d['stages'], d['kernels_rank0']['sketch_hash_ms_avg'])"
done
