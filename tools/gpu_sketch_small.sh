#!/bin/bash
# Sketch stage at 1/8 of configs[1] (125 genomes, one rank's share at 8 GPUs): kernel trace per step.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out/sk
for g in 125 1000; do
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sk/g$g -o t -- python bench.py --genomes $g --steps 5 --warmup 2 --cpu-baseline 0 --check 0 > gpurun_out/sk/g$g.json 2> gpurun_out/sk/g$g.err || exit 1
f=$(find gpurun_out/sk/g$g -name "*kernel_stats.csv" | head -1)
echo "genomes=$g"; python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:8]: print('  %-60s calls %5s avg %.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
done
