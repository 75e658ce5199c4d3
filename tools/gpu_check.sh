#!/bin/bash
# One GPU-box pass over the round's checks (run from the repo root):
#   host CPU share probe, the default bench (configs[1]), the bench with
#   --gpus 2 (two ranks started by bench.py itself, gloo sharing the one GPU,
#   --verify 1), then the GPU test suite (tools/gpu_tests.sh).
# SKIP_TESTS=1 skips the suite; TESTS / pytest args pass through to it.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
python3 - > gpurun_out/cpu_share.json <<'EOF'
import json, os
q = None
try:
    q = open("/sys/fs/cgroup/cpu.max").read().strip()
except OSError:
    pass
print(json.dumps({"affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(), "cgroup_cpu_max": q,
                  "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}))
EOF
cat gpurun_out/cpu_share.json
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('gpurun_out/bench.json'))
print('bench', d['ms_per_step'], d['value'], d['dist_pairs_per_s'], d['verified'], json.dumps(d['cpu_baseline'])[:600])"
DREPHIP_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --verify 1 --cpu-baseline 0 \
    > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err || { echo "bench --gpus 2 failed"; tail -20 gpurun_out/bench_g2.err; exit 1; }
python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/bench_g2.json') if l.startswith('{')][-1])
print('bench --gpus 2', d['n_gpus'], d['ranks_seen'], d['backend'], d.get('verified_against_single_gpu'), d['verified'], d['ms_per_step'])"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
    bash tools/gpu_tests.sh "$@" || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/gputest.log | head -30; exit 1; }
fi
