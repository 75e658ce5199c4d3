#!/bin/bash
# linkage parity (both chain implementations) + timings: cached-NN vs scan
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -v -k "linkage or cluster_mash" --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_link.log 2>&1 || { tail -40 gpurun_out/gpu_link.log; exit 1; }
tail -2 gpurun_out/gpu_link.log
for n in 10000 30000; do
  timeout -k 10 300 python3 tools/link_bench.py $n average 1 >> gpurun_out/link_bench.jsonl || exit 1
  DREPHIP_LINK_IMPL=scan timeout -k 10 300 python3 tools/link_bench.py $n average 0 >> gpurun_out/link_bench.jsonl || exit 1
done
cat gpurun_out/link_bench.jsonl
