#!/bin/bash
# Round-5 final state: the whole GPU suite (scale JSONs included), then smoke().
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.txt 2>&1 \
    || { tail -30 $O/gputest.txt; exit 1; }
tail -3 $O/gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -5 $O/smoke.txt
