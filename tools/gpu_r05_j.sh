#!/bin/bash
# Descending screened column lists A/B at configs[4] (DREPHIP_SCREEN_DESC),
# then the world-8 rehearsal and the dense one-species set (tools/gpu_r05_c.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05desc
mkdir -p $O
i=0
for V in 1 0 1 0; do
  i=$((i+1))
  DREPHIP_SCREEN_DESC=$V timeout -k 10 300 python -u bench.py --genomes 10000 --sketch 10000 \
      --steps 3 --warmup 1 --check 0 --cpu-baseline 0 > $O/b_$i.json 2> $O/b_$i.err || { echo "desc $V failed"; tail -5 $O/b_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b_$i.json')); k=d['kernels_rank0']
print('desc $V: allpairs %.2f ms, screen %.2f ms, step %.1f ms' % (k['allpairs_ms_avg'], k['screen_ms_avg'], d['ms_per_step']))" \
      | tee -a $O/summary.txt
done
bash tools/gpu_r05_c.sh
