#!/bin/bash
# All-pairs kernel profiles on the GPU box (run from the repo root): per case a
# kernel trace (average dispatch time), the HBM traffic passes (FETCH_SIZE,
# WRITE_SIZE: separate passes, MI355X_MICROARCH.md HBM), an L2 pass
# (TCC_HIT_sum / TCC_MISS_sum) and three SQ issue/stall passes, each its own
# rocprofv3 run; then tools/allpairs_traffic_json.py writes one summary per
# case.  CASES picks a subset (default: all).  Every profiled command runs the
# product path only (no oracle work under the profiler).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
R=${ROUND:-r03}
OUT=$PWD/gpurun_out/$R/ap
mkdir -p $OUT
BARGS="--check 0 --cpu-baseline 0"
CGROUPS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
         "FETCH_SIZE GRBM_GUI_ACTIVE"
         "WRITE_SIZE GRBM_GUI_ACTIVE"
         "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE")
prof() {   # name kernel-substring N s calls limit command...  (FAM: the generator's family size)
  local name=$1 key=$2 n=$3 sk=$4 nc=$5 lim=$6; shift 6
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${name}_trace -o t -- "$@" \
      > $OUT/${name}_trace.log 2>&1 || { echo "$name trace failed"; tail -5 $OUT/${name}_trace.log; return 1; }
  local i=0
  for grp in "${CGROUPS[@]}"; do
    i=$((i+1))
    timeout -s KILL $lim rocprofv3 --pmc $grp --output-format csv -d $OUT/${name}_p$i -o pmc -- "$@" \
        > $OUT/${name}_p$i.log 2>&1 || { echo "$name pass $i failed"; tail -5 $OUT/${name}_p$i.log; return 1; }
  done
  python3 tools/allpairs_traffic_json.py $key $OUT $name $n $sk $nc ${FAM:-100} > $OUT/${name}.json || return 1
  echo "$name done"
}
want() { [ -z "$CASES" ] || [[ " $CASES " == *" $1 "* ]]; }
want N1000 && { prof N1000 k_allpairs_q 1000 1000 4 180 python bench.py --steps 1 --warmup 0 $BARGS || exit 1; }
want N6000 && { AP_N=6000 AP_L=5000000 AP_ITERS=1 AP_SAMPLE=1000 prof N6000 k_allpairs_q 6000 1000 1 180 python tools/ap_bench.py || exit 1; }
want N10000 && { prof N10000 k_allpairs_q 10000 1000 4 240 python bench.py --genomes 10000 --steps 1 --warmup 0 $BARGS || exit 1; }
want N100000 && { AP_N=100000 AP_L=2000000 AP_ITERS=1 AP_SAMPLE=1000 prof N100000 k_allpairs_q 100000 1000 1 300 python tools/ap_bench.py || exit 1; }
want N10000_dense && { FAM=10000 prof N10000_dense k_allpairs_q 10000 1000 4 240 python bench.py --genomes 10000 --family-size 10000 --steps 1 --warmup 0 $BARGS || exit 1; }
want N10000_s10000 && { prof N10000_s10000 k_allpairs_band 10000 10000 4 300 python bench.py --genomes 10000 --sketch 10000 --steps 1 --warmup 0 $BARGS || exit 1; }
echo "profiles in $OUT"
