#!/bin/bash
# SQ counter passes of tools/ap_bench.py for each library in AB_LIBS (A/B of
# the all-pairs kernel): one pass per counter group, then a summary per lib.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
N=${AP_N:-6000}
OUT=$PWD/gpurun_out/appmc
mkdir -p $OUT
CGROUPS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE")
for v in ${AB_LIBS}; do
  i=0
  for grp in "${CGROUPS[@]}"; do
    i=$((i+1))
    DREPHIP_LIB=$PWD/drep_amd/lib_ab/$v/libdrephip.so AP_ITERS=1 AP_SAMPLE=1000 AP_N=$N timeout -s KILL 120 \
        rocprofv3 --pmc $grp --output-format csv -d $OUT/${v}_sq$i -o pmc -- python tools/ap_bench.py \
        > $OUT/${v}_sq$i.log 2>&1 || { echo "pmc $v $i failed"; tail -5 $OUT/${v}_sq$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py k_allpairs_q $OUT/${v}_sq*/pmc_counter_collection.csv > $OUT/$v.json || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/$v.json')); c=d['counters']; print('$v', {k: '%.3g' % v for k, v in c.items()}); print('$v', d['derived'])"
done
