#!/bin/bash
# The light screen at configs[2] (s = 1000, q LIST kernel): A/B of the bench line;
# one rank's screened stage at configs[4] for an 8-way job (tools/rank_screen.py).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05t
mkdir -p $O
i=0
for V in 1 0 1 0; do
  i=$((i+1))
  DREPHIP_SCREEN_LIGHT=$V DREPHIP_SCREEN_PROF=1 timeout -k 10 300 python -u bench.py --genomes 10000 --steps 3 --warmup 1 \
      --check 0 --cpu-baseline 0 > $O/c2_$i.json 2> $O/c2_$i.err || { echo "c2 light $V failed"; tail -5 $O/c2_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/c2_$i.json')); k=d['kernels_rank0']; sc=d['dist_kernel']['screen']
print('configs[2] light $V: allpairs %.3f ms, screen %.3f ms, step %.2f ms, marked %d, written by screen %d' % (k['allpairs_ms_avg'], k['screen_ms_avg'], d['ms_per_step'], sc['marked'], sc['simple']))" | tee -a $O/summary.txt
  grep "screen phases" $O/c2_$i.err | tail -1 >> $O/summary.txt
done
RS_N=10000 RS_S=10000 RS_W=8 timeout -k 10 400 python -u tools/rank_screen.py > $O/rank_screen_c4_w8.json 2> $O/rank_screen.err \
    || { tail -5 $O/rank_screen.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/rank_screen_c4_w8.json')); w=d['whole']
print('whole: screen %.2f ms, list %.2f ms' % (w['screen_ms'], w['list_kernel_ms']))
for r in d['ranges']: print('rows', r['rows'], 'screen %.2f ms, list %.2f ms, marked %d' % (r['screen_ms'], r['list_kernel_ms'], r['marked']))" | tee -a $O/summary.txt
