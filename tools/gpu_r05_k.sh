#!/bin/bash
# Per-wave partials A/B (default vs blockparts vs prevdiv), linkage suite first,
# then the chain's diagnostic counts at 10^5 (the known merges by kind).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT_DIR=r05link7 VARIANTS="default blockparts prevdiv default blockparts" bash tools/gpu_link_ab.sh || exit 1
DREPHIP_LIB=drep_amd/lib_ab/diag/libdrephip.so timeout -k 10 300 python tools/link_ab.py 100000 \
    > gpurun_out/r05link7/diag.json 2> gpurun_out/r05link7/diag.err || { tail -5 gpurun_out/r05link7/diag.err; exit 1; }
grep "chain" gpurun_out/r05link7/diag.err | sort -u | tee -a gpurun_out/r05link7/summary.txt
