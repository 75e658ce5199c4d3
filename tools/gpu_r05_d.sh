#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT_DIR=r05link4 PHASES=1 VARIANTS="default nodefer env:DREPHIP_LINK_SPEC=2 prevr5 default nodefer" \
    bash tools/gpu_link_ab.sh && bash tools/gpu_r05_sketch_ablate.sh
