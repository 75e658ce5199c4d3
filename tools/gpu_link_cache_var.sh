#!/bin/bash
# Per-launch cost of the cached chain's parts: variants built by tools/build_ab.sh
# (lkc_nocr: caches never read -- same launches as the plain step;
#  lkc_nocr_noref: and no refresh; lkc_bare: and no maintenance), chain at N = 10^4.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/lkvar
for v in ${VARS:-lib lkc_nocr lkc_bare}; do
  if [ "$v" = lib ]; then L=$PWD/drep_amd/lib/libdrephip.so; else L=$PWD/drep_amd/lib_ab/$v/libdrephip.so; fi
  DREPHIP_DEBUG=1 LINK_AB_TIMING_ONLY=1 DREPHIP_LINK_CACHE=1 DREPHIP_LIB=$L timeout -k 10 300 python tools/link_ab.py ${N:-10000} > gpurun_out/lkvar/$v.json 2> gpurun_out/lkvar/$v.err || { echo "$v failed"; tail -3 gpurun_out/lkvar/$v.err; exit 1; }
  echo "$v: $(grep 'cached chain' gpurun_out/lkvar/$v.err | tail -1)"
  python3 -c "import json; d=json.load(open('gpurun_out/lkvar/$v.json')); print('   chain ms', round(d['chain_kernel_ms_0'],1), round(d['chain_kernel_ms_1'],1), 'scipy', d['Z_equals_scipy_digest'])"
done
