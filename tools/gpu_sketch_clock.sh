#!/bin/bash
# Effective clock of the sketch kernel at 125 vs 1000 genomes (GRBM_GUI_ACTIVE per dispatch / duration).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out/skc
for g in 125 1000; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/skc/g$g -o pmc -- python bench.py --genomes $g --steps 5 --warmup 2 --cpu-baseline 0 --check 0 > gpurun_out/skc/g$g.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/skc/t$g -o t -- python bench.py --genomes $g --steps 5 --warmup 2 --cpu-baseline 0 --check 0 > gpurun_out/skc/t$g.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for g in (125, 1000):
    f = glob.glob('gpurun_out/skc/g%d/**/*counter_collection.csv' % g, recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if 'k_sketch_hash21' in r['Kernel_Name']]
    c = collections.defaultdict(list)
    for r in rows: c[r['Counter_Name']].append(float(r['Counter_Value']))
    t = glob.glob('gpurun_out/skc/t%d/**/*kernel_trace.csv' % g, recursive=True)[0]
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) for r in csv.DictReader(open(t)) if 'k_sketch_hash21' in r['Kernel_Name']]
    gui = sorted(c['GRBM_GUI_ACTIVE'])
    print(g, 'GUI_ACTIVE per dispatch (sorted)', [round(x / 1e6, 3) for x in gui], 'Mcyc; durations us', [round(x / 1e3) for x in d])
PY
