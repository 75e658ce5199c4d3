#!/bin/bash
# Linkage: the Markstein division A/B against the previous kernel (prevdiv),
# the linkage suite first; then the configs[4] whole-triangle check and the
# LIST kernel profile with the light screen (tools/gpu_r05_g.sh, second part).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT_DIR=r05link6 VARIANTS="default prevdiv default prevdiv" bash tools/gpu_link_ab.sh || exit 1
O=gpurun_out/r05light
mkdir -p $O
DREPHIP_SCALE_ONLY=10000-s10000 timeout -k 10 900 python -u -m pytest tests/test_scale.py -m gpu -x -q --timeout 880 \
    --timeout-method thread > $O/scale_s10000.log 2>&1 || { tail -30 $O/scale_s10000.log; exit 1; }
tail -1 $O/scale_s10000.log | tee -a $O/summary.txt
ROUND=r05 CASES=N10000_s10000 bash tools/profile_allpairs.sh || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r05/ap/N10000_s10000.json')); dv=d['derived']
print('profile light: ms %.2f' % d['avg_call_ms'], 'l2 hit %.3f' % dv['l2_hit_rate'], 'hbm/alg %.1f' % dv['hbm_over_algorithmic_x2'])" | tee -a $O/summary.txt
