#!/bin/bash
# With the light screen, the band LIST kernel streams family (heavy) cells only:
# value rounds A/B again at configs[4] (DREPHIP_BAND_ROUND 0 / 1280 / 640).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
OUT_DIR=r05band2 SKIP_TESTS=1 ROUNDS="0 1280 640 0 1280 640" bash tools/gpu_r05_band.sh
