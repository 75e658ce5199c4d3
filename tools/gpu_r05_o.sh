#!/bin/bash
# Fused known merges: the linkage suite, then same-box chain A/B against the
# unfused protocol (DREPHIP_LINK_FUSE=0), Z digest vs scipy, and the diagnostic counts.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT_DIR=r05link9 VARIANTS="default env:DREPHIP_LINK_FUSE=0 default env:DREPHIP_LINK_FUSE=0" bash tools/gpu_link_ab.sh || exit 1
DREPHIP_LIB=drep_amd/lib_ab/diag/libdrephip.so timeout -k 10 300 python tools/link_ab.py 100000 \
    > gpurun_out/r05link9/diag.json 2> gpurun_out/r05link9/diag.err || { tail -5 gpurun_out/r05link9/diag.err; exit 1; }
grep "chain" gpurun_out/r05link9/diag.err | sort -u | tee -a gpurun_out/r05link9/summary.txt
