#!/bin/bash
# Candidate-row prefetch chain A/B (linkage suite first), then the band
# kernel's value rounds profiled at configs[4] (no rounds vs 640 elements per
# round): L2 hit rate and HBM traffic (tools/profile_allpairs.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT_DIR=r05link5 PHASES=1 VARIANTS="default nopf prevr5 env:DREPHIP_LINK_SPEC=3 pfdefer default nopf" \
    bash tools/gpu_link_ab.sh || exit 1
DREPHIP_BAND_ROUND=0 ROUND=r05 CASES=N10000_s10000 bash tools/profile_allpairs.sh || exit 1
DREPHIP_BAND_ROUND=640 ROUND=r05rd CASES=N10000_s10000 bash tools/profile_allpairs.sh || exit 1
for r in r05 r05rd; do python3 -c "
import json; d=json.load(open('gpurun_out/$r/ap/N10000_s10000.json')); dv=d['derived']
print('$r', 'ms %.2f' % d['avg_call_ms'], 'l2 hit %.3f' % dv['l2_hit_rate'], 'hbm/alg %.1f' % dv['hbm_over_algorithmic_x2'], 'valu %.2f lds %.2f' % (dv['valu_issue_frac_2cyc'], dv['lds_busy_frac']))"; done
