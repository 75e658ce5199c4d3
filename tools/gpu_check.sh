#!/bin/bash
# GPU-box check during development: optional microbench, parity tests (incl.
# the configs[2]/[3] scale tests), smoke, then the default bench.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
if [ -x tools/lds_microbench ] && [ -n "$LDS_MB" ]; then
  timeout -k 10 120 tools/lds_microbench > gpurun_out/lds_microbench.json 2>&1 || { echo "lds microbench failed"; cat gpurun_out/lds_microbench.json; exit 1; }
  cat gpurun_out/lds_microbench.json
fi
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
