#!/bin/bash
# Collects the round's profiles on the GPU box (run from the repo root):
#   kernel trace + stats of the default bench, and HBM traffic PMC passes
#   (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md HBM).
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
