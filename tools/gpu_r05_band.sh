#!/bin/bash
# Band kernel value rounds (round 5): the all-pairs GPU tests, then a same-box
# A/B of the round size (DREPHIP_BAND_ROUND; 0 = no rounds) at configs[4]
# (10^4 genomes, s = 10^4, screened LIST kernel) from bench.py's live HIP-event
# kernel times, interleaved.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${OUT_DIR:-r05band}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "allpairs" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log | tee -a $O/summary.txt
fi
i=0
for V in ${ROUNDS:-0 640 320 1280 640 0}; do
  i=$((i+1))
  DREPHIP_BAND_ROUND=$V timeout -k 10 300 python -u bench.py --genomes 10000 --sketch 10000 --steps 3 --warmup 1 \
      --check 0 --cpu-baseline 0 > $O/b_$i.json 2> $O/b_$i.err || { echo "round $V failed"; tail -5 $O/b_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b_$i.json')); k=d['kernels_rank0']
print('round $V: allpairs %.2f ms, screen %.2f ms, step %.1f ms' % (k['allpairs_ms_avg'], k['screen_ms_avg'], d['ms_per_step']))" \
      | tee -a $O/summary.txt
done
