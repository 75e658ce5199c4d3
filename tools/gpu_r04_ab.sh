#!/bin/bash
# Round-4 A/B pass on the box (run from the repo root):
#   1. GPU tests of the sketch sizes above 12000, the finalize and the band kernel
#   2. k_allpairs_q with 4 vs 8 rows per workgroup (DREPHIP_AP_R; 8 = one
#      160 KiB workgroup per CU) at N = 6000 and 10^4, whole triangle checked
#   3. the band kernel with live column lists vs round 3's (lib_ab/band_r3)
#      at configs[4] (N = 10^4, s = 10^4)
#   4. linkage: column-y stores plain / nontemporal / none (timing only)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "sketch_sizes or finalize or band or errors_are" > gpurun_out/ab/tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
for n in 6000 10000; do
  timeout -k 10 300 python tools/ap_ab.py $n 4,8 3 > gpurun_out/ab/q_$n.json 2> gpurun_out/ab/q_$n.err \
      || { echo "ap_ab $n failed"; tail -20 gpurun_out/ab/q_$n.err; exit 1; }
  grep round gpurun_out/ab/q_$n.err
done
for v in lib band_r3 lib band_r3; do
  if [ "$v" = lib ]; then L=$PWD/drep_amd/lib/libdrephip.so; else L=$PWD/drep_amd/lib_ab/$v/libdrephip.so; fi
  DREPHIP_LIB=$L AB_S=10000 timeout -k 10 300 python tools/ap_ab.py 10000 "" 2 > gpurun_out/ab/band_$v.json 2> gpurun_out/ab/band_$v.err \
      || { echo "band $v failed"; tail -20 gpurun_out/ab/band_$v.err; exit 1; }
  echo "band $v:"; grep round gpurun_out/ab/band_$v.err
done
AB_LIBS="lk_base lk_ntcol lk_nocol" LINK_NS="10000 100000" bash tools/gpu_link_ab.sh
