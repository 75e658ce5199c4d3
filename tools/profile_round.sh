#!/bin/bash
# Collects the round's profiles on the GPU box (run from the repo root):
#   kernel trace + stats of the default bench, HBM traffic PMC passes
#   (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md HBM),
#   and SQ issue/stall counter passes (<= 8 SQ + 2 GRBM counters per pass).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
R=${ROUND:-r01}
OUT=$PWD/gpurun_out/$R
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
    python bench.py --steps 5 --warmup 1 --cpu-baseline 0 > $OUT/trace_bench.json 2> $OUT/trace.err || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o pmc -- \
      python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || exit 1
done
python3 tools/traffic_json.py $OUT ${GENOMES:-1000} ${GENOME_BP:-5000000} > $OUT/sketch_traffic.json || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq$i -o pmc -- \
      python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/sq$i.json 2> $OUT/sq$i.err || exit 1
done
python3 tools/pmc_summary.py k_sketch_hash21 $OUT/sq*/pmc_counter_collection.csv > $OUT/sketch_pmc_sq.json || exit 1
python3 tools/pmc_summary.py k_allpairs_q $OUT/sq*/pmc_counter_collection.csv > $OUT/allpairs_pmc_sq_N1000.json || exit 1
