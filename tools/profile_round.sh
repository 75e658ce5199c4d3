#!/bin/bash
# Collects the round's profiles on the GPU box (run from the repo root):
#   kernel trace + stats of the default bench, HBM traffic PMC passes
#   (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md HBM),
#   SQ issue/stall counter passes (<= 8 SQ + 2 GRBM counters per pass) of the
#   bench (sketch kernel).  The all-pairs kernel's passes are
#   tools/profile_allpairs.sh.  Every profiled command runs the product path only
#   (--check 0 --cpu-baseline 0: no oracle work under the profiler).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
R=${ROUND:-r03}
OUT=$PWD/gpurun_out/$R
mkdir -p $OUT
BARGS="--check 0 --cpu-baseline 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
    python bench.py --steps 5 --warmup 1 $BARGS > $OUT/trace_bench.json 2> $OUT/trace.err || exit 1
KMS=$(python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/trace/**/*kernel_stats.csv', recursive=True)[0])):
    if 'k_sketch_hash21' in r['Name']: print(float(r['AverageNs'])/1e6)
") || exit 1
echo "sketch hash kernel avg ms under rocprof: $KMS"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o pmc -- \
      python bench.py --steps 1 --warmup 0 $BARGS > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || exit 1
done
python3 tools/traffic_json.py $OUT ${GENOMES:-1000} ${GENOME_BP:-5000000} > $OUT/sketch_traffic.json || exit 1
WE=$(python3 -c "print(${GENOMES:-1000} * ((${GENOME_BP:-5000000} + 1 + 32767) // 32768 * 32768))")
CGROUPS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
        "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE")
i=0
for grp in "${CGROUPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq$i -o pmc -- \
      python bench.py --steps 1 --warmup 0 $BARGS > $OUT/sq$i.json 2> $OUT/sq$i.err || exit 1
done
python3 tools/pmc_summary.py k_sketch_hash21 $OUT/sq*/pmc_counter_collection.csv --window-ends $WE --kernel-ms $KMS \
    > $OUT/sketch_pmc_sq.json || exit 1
echo "profiles in $OUT"
