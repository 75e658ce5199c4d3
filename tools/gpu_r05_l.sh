#!/bin/bash
# tools/gpu_r05_k.sh (per-wave partials A/B, chain diagnostics) then
# tools/gpu_r05_j.sh (descending lists A/B, world-8 rehearsal, dense set).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/gpu_r05_k.sh && bash tools/gpu_r05_j.sh
