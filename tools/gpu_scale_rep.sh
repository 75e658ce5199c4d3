#!/bin/bash
# repeat the N=20000 scale test (wrong-result hunt; no GPU fault involved)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3 4; do
  DREPHIP_SCALE_N=${N:-20000} DREPHIP_SCALE_OUT=gpurun_out/scale_rep$rep.json timeout -k 10 300 python -u -m pytest tests/test_scale.py -m gpu -x -q -s \
      --timeout 280 --timeout-method thread > gpurun_out/scale_rep$rep.log 2>&1
  rc=$?
  echo "rep $rep rc $rc"; grep -E "second pass|parity|passed|failed" gpurun_out/scale_rep$rep.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
