#!/bin/bash
# All-pairs with row-group LDS images: parity tests, timings at N = 1000 / 6000,
# rank 0's shard step of the 8-way job, and the default bench.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/apimg
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/apimg/tests.log 2>&1 || { tail -40 gpurun_out/apimg/tests.log; exit 1; }
tail -1 gpurun_out/apimg/tests.log
for N in 1000 6000 20000; do
  AP_N=$N AP_S=1000 AP_PATH=table AP_L=5000000 AP_SAMPLE=20000 timeout -k 10 200 python tools/ap_bench.py 2>/dev/null > gpurun_out/apimg/ap_$N.json || { echo "ap $N failed"; exit 1; }
  echo "N=$N: $(cat gpurun_out/apimg/ap_$N.json)"
done
SHARD_TIMING=1 timeout -k 10 120 python tools/shard_step.py 1000 8 0 50 || exit 1
SHARD_TIMING=0 timeout -k 10 120 python tools/shard_step.py 1000 8 0 50 || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/apimg/bench.json 2>/dev/null || exit 1
python -c "
import json; d=json.load(open('gpurun_out/apimg/bench.json')); print(d['ms_per_step'], d['value'], d['kernels_rank0'])"
