#!/bin/bash
# GPU-box check used during development: parity tests, then the default bench.
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; exit 1; }
