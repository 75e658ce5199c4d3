#!/bin/bash
# Chain-step grid density at 10^5 after the DPP / two-step changes: entries per lane 1, 2 (default), 4.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/lkd
for pl in 2 1 4 2; do
  DREPHIP_LINK_PER_LANE=$pl timeout -k 10 300 python tools/link_ab.py ${N:-100000} > gpurun_out/lkd/pl$pl.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/lkd/pl$pl.json')); print('per_lane=$pl chain ms %.1f / %.1f' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'scipy', d['Z_equals_scipy_digest'])"
done
