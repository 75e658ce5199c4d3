#!/bin/bash
# World-8 rehearsal (tools/gpu_r05_world8.sh), then the dense one-species set
# at configs[2] size (tests/test_scale.py::test_scale[10000-dense]) and the
# bench line on it (family size = N: every pair related).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/gpu_r05_world8.sh || exit 1
mkdir -p gpurun_out/r05c
DREPHIP_SCALE_ONLY=10000-dense timeout -k 10 600 python -u -m pytest tests/test_scale.py -m gpu -x -q --timeout 560 \
    --timeout-method thread > gpurun_out/r05c/scale_dense.log 2>&1 || { tail -30 gpurun_out/r05c/scale_dense.log; exit 1; }
tail -2 gpurun_out/r05c/scale_dense.log
timeout -k 10 300 python -u bench.py --genomes 10000 --family-size 10000 --steps 5 --warmup 2 --cpu-baseline 0 \
    > gpurun_out/r05c/bench_dense_10000.json 2> gpurun_out/r05c/bench_dense_10000.err || { tail -20 gpurun_out/r05c/bench_dense_10000.err; exit 1; }
tail -c 600 gpurun_out/r05c/bench_dense_10000.json
