#!/bin/bash
# Round-5 measurement: the default bench line, its rocprofv3 kernel trace and
# PMC passes (tools/profile_round.sh), the 10^5 chain trace, and the value-round
# A/B with the light screen (tools/gpu_r05_r.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
tail -c 400 gpurun_out/bench.json
ROUND=r05 bash tools/profile_round.sh || { echo "profile failed"; exit 1; }
N=100000 bash tools/gpu_link_trace.sh > gpurun_out/r05_trace_1e5.txt 2>&1 || { tail -20 gpurun_out/r05_trace_1e5.txt; exit 1; }
cat gpurun_out/r05_trace_1e5.txt
bash tools/gpu_r05_r.sh
