#!/bin/bash
# Parity tests, the default bench, then one rank's step of the 8-way sharded
# bench rehearsed on one GPU (with and without timing events) and a kernel
# trace of it (gaps between dispatches).
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/shard
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/shard/tests.log 2>&1 || { tail -30 gpurun_out/shard/tests.log; exit 1; }
tail -1 gpurun_out/shard/tests.log
timeout -k 10 300 python bench.py > gpurun_out/shard/bench.json 2>gpurun_out/shard/bench.err || { tail gpurun_out/shard/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/shard/bench.json')); print(d['ms_per_step'], d['value'], d['kernels_rank0'])"
for t in 1 0; do
  SHARD_TIMING=$t timeout -k 10 120 python tools/shard_step.py 1000 8 0 50 > gpurun_out/shard/step_t$t.json || exit 1
  cat gpurun_out/shard/step_t$t.json
done
SHARD_TIMING=0 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/shard/trace -o shard -- python tools/shard_step.py 1000 8 0 20 > /dev/null 2>gpurun_out/shard/trace.err || exit 1
python tools/trace_gaps.py $(find gpurun_out/shard/trace -name "shard_kernel_trace.csv") 12
