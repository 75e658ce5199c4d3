#!/bin/bash
# Round-4 profiles on the box: the sketch kernel's (tools/profile_round.sh:
# kernel trace/stats of the default bench, HBM traffic passes, SQ passes) and
# kernel traces of the screened all-pairs stage at configs[2], configs[4]
# (bench) and 10^5 genomes (tools/ap_ab.py, screen on, no reference check).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
ROUND=r04 bash tools/profile_round.sh || exit 1
OUT=$PWD/gpurun_out/r04
BARGS="--check 0 --cpu-baseline 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c2 -o t -- \
    python bench.py --genomes 10000 --steps 3 --warmup 1 $BARGS > $OUT/trace_c2.json 2> $OUT/trace_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c4 -o t -- \
    python bench.py --genomes 10000 --sketch 10000 --steps 3 --warmup 1 $BARGS > $OUT/trace_c4.json 2> $OUT/trace_c4.err || exit 1
AB_NOREF=1 AB_VAR=DREPHIP_AP_SCREEN timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_1e5 -o t -- \
    python tools/ap_ab.py 100000 1 3 > $OUT/trace_1e5.json 2> $OUT/trace_1e5.err || exit 1
# the all-pairs kernels' counter passes at configs[2] and configs[4] (screened: the LIST kernels)
CASES="N1000 N10000 N10000_s10000" ROUND=r04 bash tools/profile_allpairs.sh || exit 1
echo done
