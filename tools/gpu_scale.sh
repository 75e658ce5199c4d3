#!/bin/bash
# configs[3]-style single-GPU scale run (tests/test_scale.py), chained so a
# failing step ends the call.  usage: bash tools/gpu_scale.sh "20000:1 100000:0"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "allpairs" --timeout 120 --timeout-method thread \
    > gpurun_out/scale_pre_tests.log 2>&1 || { tail -30 gpurun_out/scale_pre_tests.log; exit 1; }
tail -1 gpurun_out/scale_pre_tests.log
for spec in ${1:-"20000:1 100000:0"}; do
  n=${spec%%:*}; sc=${spec##*:}
  DREPHIP_SCALE_N=$n DREPHIP_SCALE_SCIPY=$sc timeout -k 10 1000 python -u -m pytest tests/test_scale.py -m gpu -x -v -s \
      --timeout 1000 --timeout-method thread > gpurun_out/scale_$n.log 2>&1 || { tail -30 gpurun_out/scale_$n.log; exit 1; }
  grep -E "allpairs|second|parity|linkage" gpurun_out/scale_$n.log; tail -1 gpurun_out/scale_$n.log
done
