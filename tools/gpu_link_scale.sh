#!/bin/bash
# linkage parity, then 10^5 scale runs at several grid densities (entries per lane)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "linkage or cluster_mash" --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_link.log 2>&1 || { tail -40 gpurun_out/gpu_link.log; exit 1; }
tail -1 gpurun_out/gpu_link.log
for per in ${PERS:-4 1}; do
  DREPHIP_LINK_PER_LANE=$per DREPHIP_SCALE_N=${N:-100000} DREPHIP_SCALE_OUT=gpurun_out/scale_link_$per.json timeout -k 10 600 \
     python -u -m pytest tests/test_scale.py -m gpu -x -q -s --timeout 580 --timeout-method thread > gpurun_out/scale_link_$per.log 2>&1 \
     || { tail -20 gpurun_out/scale_link_$per.log; exit 1; }
  echo "per lane $per"; grep -o '"linkage_s[^}]*' gpurun_out/scale_link_$per.log | tail -1
done
