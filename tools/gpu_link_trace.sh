#!/bin/bash
# Chain launch count (DREPHIP_DEBUG) and rocprofv3 kernel trace of tools/link_ab.py at N.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out/lktr
DREPHIP_DEBUG=1 timeout -k 10 300 python tools/link_ab.py ${N:-10000} > gpurun_out/lktr/run.json 2> gpurun_out/lktr/run.err || exit 1
grep "chain:" gpurun_out/lktr/run.err | tail -3
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lktr/tr -o t -- python tools/link_ab.py ${N:-10000} > gpurun_out/lktr/tr.log 2>&1 || exit 1
f=$(find gpurun_out/lktr/tr -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, numpy as np, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows: d[r['Kernel_Name'][:40]].append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
for k, v in d.items():
    if len(v) < 1000: continue
    v.sort(); dur = np.array([e - s for s, e in v]); st = np.array([s for s, e in v])
    gap = st[1:] - np.array([e for s, e in v])[:-1]
    print(k, len(v), "dur med %.2f us p90 %.2f" % (np.median(dur) / 1e3, np.percentile(dur, 90) / 1e3),
          "gap med %.2f us p90 %.2f" % (np.median(gap) / 1e3, np.percentile(gap, 90) / 1e3))
PY
rm -rf gpurun_out/lktr/tr                                  # (the trace CSV: tens of MB)
