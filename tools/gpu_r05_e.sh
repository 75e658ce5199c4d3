#!/bin/bash
# Deferral / spec-4 chain A/B and the sketch ablation (gpu_r05_d.sh), then the
# band kernel's value-round tests and A/B (gpu_r05_band.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/gpu_r05_d.sh && bash tools/gpu_r05_band.sh
