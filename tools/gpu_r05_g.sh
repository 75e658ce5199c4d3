#!/bin/bash
# Light screen (k_screen_light): the screen and all-pairs GPU tests, a same-box
# A/B at configs[4] (DREPHIP_SCREEN_LIGHT 1 vs 0: screen, LIST kernel and step
# times), the configs[4] whole-triangle check (tests/test_scale.py), then the
# LIST kernel's profile at configs[4] (tools/profile_allpairs.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05light
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_screen.py tests/test_gpu.py \
    -k "screen or allpairs" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log | tee -a $O/summary.txt
i=0
for V in 1 0 1 0; do
  i=$((i+1))
  DREPHIP_SCREEN_LIGHT=$V DREPHIP_SCREEN_PROF=1 timeout -k 10 300 python -u bench.py --genomes 10000 --sketch 10000 \
      --steps 3 --warmup 1 --check 0 --cpu-baseline 0 > $O/b_$i.json 2> $O/b_$i.err || { echo "light $V failed"; tail -5 $O/b_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b_$i.json')); k=d['kernels_rank0']; sc=d['dist_kernel']['screen']
print('light $V: allpairs %.2f ms, screen %.2f ms, step %.1f ms, marked %d, written by screen %d' % (k['allpairs_ms_avg'], k['screen_ms_avg'], d['ms_per_step'], sc['marked'], sc['simple']))" \
      | tee -a $O/summary.txt
  grep "screen phases" $O/b_$i.err | tail -1 >> $O/summary.txt
done
[ "${LIGHT_ONLY_AB:-0}" = 1 ] && exit 0
DREPHIP_SCALE_ONLY=10000-s10000 timeout -k 10 900 python -u -m pytest tests/test_scale.py -m gpu -x -q --timeout 880 \
    --timeout-method thread > $O/scale_s10000.log 2>&1 || { tail -30 $O/scale_s10000.log; exit 1; }
tail -1 $O/scale_s10000.log | tee -a $O/summary.txt
ROUND=r05 CASES=N10000_s10000 bash tools/profile_allpairs.sh || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r05/ap/N10000_s10000.json')); dv=d['derived']
print('profile light: ms %.2f' % d['avg_call_ms'], 'l2 hit %.3f' % dv['l2_hit_rate'], 'hbm/alg %.1f' % dv['hbm_over_algorithmic_x2'])" | tee -a $O/summary.txt
