#!/bin/bash
# linkage pass 2, then the sketch kernel's binding-resource ablation
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/gpu_r05_link2.sh && bash tools/gpu_r05_sketch_ablate.sh
