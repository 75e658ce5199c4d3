#!/bin/bash
# Round-end refresh on the GPU box: parity tests, smoke, the 8-way rank-0
# shard-step rehearsal, the round's rocprof profiles, then the default bench.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
SHARD_TIMING=0 timeout -k 10 120 python tools/shard_step.py 1000 8 0 30 > gpurun_out/shard.json 2>/dev/null || { echo "shard failed"; exit 1; }
SHARD_TIMING=1 timeout -k 10 120 python tools/shard_step.py 1000 8 0 30 >> gpurun_out/shard.json 2>/dev/null || { echo "shard failed"; exit 1; }
cat gpurun_out/shard.json
bash tools/profile_round.sh || { echo "profile failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
