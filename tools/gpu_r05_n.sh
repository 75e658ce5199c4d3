#!/bin/bash
# The step kernel with the row-y race fixed: linkage suite and chain timing at
# 10^4 / 10^5 (Z digest vs scipy), then the world-8 rehearsal and the dense set.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT_DIR=r05link8 VARIANTS="default default" bash tools/gpu_link_ab.sh || exit 1
bash tools/gpu_r05_c.sh
