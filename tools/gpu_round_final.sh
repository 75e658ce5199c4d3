#!/bin/bash
# Round-end refresh on the GPU box: parity tests, smoke, the 8-way rank-0
# shard-step rehearsal, the round's sketch profiles (tools/profile_round.sh),
# the default bench, then the configs[2] and configs[4] single-GPU bench lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
TESTS_LIMIT=500 bash tools/gpu_tests.sh || { echo "tests failed"; tail -40 gpurun_out/gputest.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
SHARD_TIMING=0 timeout -k 10 120 python tools/shard_step.py 1000 8 0 30 > gpurun_out/shard.json 2>/dev/null || { echo "shard failed"; exit 1; }
cat gpurun_out/shard.json
bash tools/profile_round.sh || { echo "profile failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
timeout -k 10 300 python bench.py --genomes 10000 --steps 3 --warmup 1 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "c2 failed"; tail -5 gpurun_out/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --genomes 10000 --sketch 10000 --steps 3 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "c4 failed"; tail -5 gpurun_out/bench_c4.err; exit 1; }
python3 -c "
import json
for f in ('bench_c2', 'bench_c4'):
    d = json.load(open('gpurun_out/%s.json' % f))
    print(f, d['ms_per_step'], d['value'], d['kernels_rank0']['sketch_hash_ms_avg'], d['kernels_rank0']['allpairs_ms_avg'], d['verified'])
"
