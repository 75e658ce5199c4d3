#!/bin/bash
# Candidate-row prefetch chain A/B (linkage suite first), then the light
# screen's tests and configs[4] A/B (the first part of tools/gpu_r05_g.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT_DIR=r05link5 PHASES=1 VARIANTS="default nopf prevr5 env:DREPHIP_LINK_SPEC=3 pfdefer default nopf" \
    bash tools/gpu_link_ab.sh || exit 1
LIGHT_ONLY_AB=1 bash tools/gpu_r05_g.sh
