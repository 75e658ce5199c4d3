#!/bin/bash
# Round-4 A/B pass on the box (run from the repo root):
#   1. the shared-hash screen on/off (DREPHIP_AP_SCREEN 2 = off, 1 = on) at
#      N = 1000 / 6000 / 10^4 / 10^5 (s = 1000) and configs[4] (10^4, s = 10^4),
#      whole triangle checked against the literal merge kernel; the screen's
#      own time (kernel_ms(4)) is part of each total
#   2. the band kernel with live column lists vs round 3's (lib_ab/band_r3), screen off
#   3. linkage: column-y stores plain / nontemporal / none (timing only)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/ab
for ns in ${SCREEN_CASES:-"1000 1000" "6000 1000" "10000 1000" "10000 10000" "100000 1000"}; do
  set -- $ns
  AB_VAR=DREPHIP_AP_SCREEN AB_S=$2 timeout -k 10 300 python tools/ap_ab.py $1 2,1 3 > gpurun_out/ab/screen_$1_$2.json 2> gpurun_out/ab/screen_$1_$2.err \
      || { echo "screen $ns failed"; tail -20 gpurun_out/ab/screen_$1_$2.err; exit 1; }
  echo "screen N=$1 s=$2:"; grep -E "round|stats" gpurun_out/ab/screen_$1_$2.err | tail -4
done
if [ "${SKIP_BAND:-0}" != 1 ]; then
for v in lib band_r3 lib band_r3; do
  if [ "$v" = lib ]; then L=$PWD/drep_amd/lib/libdrephip.so; else L=$PWD/drep_amd/lib_ab/$v/libdrephip.so; fi
  DREPHIP_AP_SCREEN=2 DREPHIP_LIB=$L AB_S=10000 timeout -k 10 300 python tools/ap_ab.py 10000 "" 2 > gpurun_out/ab/band_$v.json 2> gpurun_out/ab/band_$v.err \
      || { echo "band $v failed"; tail -20 gpurun_out/ab/band_$v.err; exit 1; }
  echo "band $v:"; grep round gpurun_out/ab/band_$v.err
done
fi
if [ "${SKIP_LINK:-0}" != 1 ]; then
AB_LIBS="lk_base lk_ntcol lk_nocol" LINK_NS="10000 100000" bash tools/gpu_link_ab.sh
fi
