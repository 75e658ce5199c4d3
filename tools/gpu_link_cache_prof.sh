#!/bin/bash
# Kernel trace of the linkage chain (tools/link_ab.py at N) for both step kernels.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out/lkprof
for c in 1 0; do
  DREPHIP_LINK_CACHE=$c timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lkprof/c$c -o t -- python tools/link_ab.py ${N:-10000} > gpurun_out/lkprof/c$c.log 2>&1 || { echo "prof c=$c failed"; tail -5 gpurun_out/lkprof/c$c.log; exit 1; }
  f=$(find gpurun_out/lkprof/c$c -name "*kernel_stats.csv" | head -1)
  echo "cache=$c"; head -6 "$f" | cut -c1-200
done
