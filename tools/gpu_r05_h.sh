#!/bin/bash
# Light screen tests and configs[4] A/B (tools/gpu_r05_g.sh, first part), the
# linkage suite, then the 10^5 chain trace (launch count + kernel trace).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k linkage \
    > gpurun_out/r05h_link_tests.log 2>&1 || { tail -30 gpurun_out/r05h_link_tests.log; exit 1; }
tail -1 gpurun_out/r05h_link_tests.log
LIGHT_ONLY_AB=1 bash tools/gpu_r05_g.sh || exit 1
N=100000 bash tools/gpu_link_trace.sh > gpurun_out/r05h_trace_1e5.txt 2>&1 || { tail -20 gpurun_out/r05h_trace_1e5.txt; exit 1; }
cat gpurun_out/r05h_trace_1e5.txt
