#!/bin/bash
# Full pass on the box: GPU suite (incl. configs[1]-[4] scale tests), smoke,
# default bench, configs[2]/[4] bench lines, bench --gpus 2 (gloo, one GPU).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
TESTS_LIMIT=${TESTS_LIMIT:-900} bash tools/gpu_tests.sh || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/gputest.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --genomes 10000 --steps 3 --warmup 1 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "c2 failed"; tail -5 gpurun_out/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --genomes 10000 --sketch 10000 --steps 3 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "c4 failed"; tail -5 gpurun_out/bench_c4.err; exit 1; }
DREPHIP_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --verify 1 --cpu-baseline 0 > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err || { echo "g2 failed"; tail -5 gpurun_out/bench_g2.err; exit 1; }
python3 -c "
import json
for f in ('bench', 'bench_c2', 'bench_c4', 'bench_g2'):
    d = json.loads([l for l in open('gpurun_out/%s.json' % f) if l.startswith('{')][-1])
    print(f, 'ms/step %.2f' % d['ms_per_step'], 'value %.3g' % d['value'], 'dist %.3g' % (d['dist_pairs_per_s'] or 0),
          'sketch %.2f ms' % d['kernels_rank0']['sketch_hash_ms_avg'], 'ap %.3f ms' % d['kernels_rank0']['allpairs_ms_avg'],
          'screen %.3f ms' % d['kernels_rank0'].get('screen_ms_avg', 0), d['dist_kernel'].get('screen', {}).get('used'),
          'verified', d.get('verified'), d.get('verified_against_single_gpu'))
"
