#!/bin/bash
# Step-workgroup shape per matrix size, compaction off (each run at one m):
# 10^5 with 256 (default) / 512 lanes, 5 x 10^4 with 256 (default) / 128 / 512.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05w
mkdir -p $O
run() {   # N WG
  DREPHIP_LINK_COMPACT=0 DREPHIP_LINK_WG=$2 timeout -k 10 400 python -u tools/link_ab.py $1 > $O/link_$1_wg$2.json 2> $O/link_$1_wg$2.err || { tail -5 $O/link_$1_wg$2.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/link_$1_wg$2.json'))
print('n=$1 WG=$2: chain %.1f ms, %.2f us per launch, Z %s' % (d['chain_kernel_ms_1'], 1e3*d['chain_kernel_ms_1']/d['launches_1'], d['Z_sha1'][:12]))" | tee -a $O/summary.txt
}
run 100000 256 && run 100000 512 && run 50000 256 && run 50000 128 && run 50000 512 && run 25000 128 && run 25000 64 && run 25000 256
