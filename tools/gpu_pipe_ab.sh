#!/bin/bash
# A/B of the bench host loop (pipelined vs one step at a time), GPU tests first.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_t8.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_t8.log; exit 1; }
tail -1 gpurun_out/gpu_t8.log
for p in 0 1 0 1; do
  SHARD_TIMING=0 SHARD_PIPE=$p timeout -k 10 120 python tools/shard_step.py 1000 8 0 40 > gpurun_out/shard_p$p.json 2>/dev/null || { echo "shard $p failed"; exit 1; }
  cat gpurun_out/shard_p$p.json
done
for p in 0 1 0 1; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --pipeline $p --steps 10 > gpurun_out/bench_p$p.json 2> gpurun_out/bench_p$p.err || { echo "bench $p failed"; tail gpurun_out/bench_p$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_p$p.json')); print('pipe', $p, d['ms_per_step'], d['value'], d['kernels_rank0']['sketch_hash_ms_avg'], d['config']['host_loop'])"
done
