#!/bin/bash
# Round-5 final state after the SGPR-pressure changes: the whole GPU suite
# (scale JSONs included), smoke(), then the 10^5 chain trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${OUT_DIR:-r05final2}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.txt 2>&1 \
    || { tail -30 $O/gputest.txt; exit 1; }
tail -3 $O/gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
N=100000 bash tools/gpu_link_trace.sh > $O/trace_1e5.txt 2>&1 || { tail -20 $O/trace_1e5.txt; exit 1; }
cat $O/trace_1e5.txt
