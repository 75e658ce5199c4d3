#!/bin/bash
# Linkage step-kernel shape A/B: workgroup size (builds in drep_amd/lib_ab/wg<size>,
# "lib" = 256) x target workgroup count (DREPHIP_LINK_TARGET_WG), tools/link_ab.py.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/linkwg
for N in ${LINK_NS:-100000 10000}; do
  for v in ${AB_LIBS:-lib wg128 wg512}; do
    for tg in ${TARGETS:-100 200 400}; do
      if [ "$v" = lib ]; then L=$PWD/drep_amd/lib/libdrephip.so; else L=$PWD/drep_amd/lib_ab/$v/libdrephip.so; fi
      DREPHIP_LIB=$L DREPHIP_LINK_TARGET_WG=$tg DREPHIP_LINK_PATH=dense timeout -k 10 300 python tools/link_ab.py $N > gpurun_out/linkwg/$v.$tg.$N.json 2> gpurun_out/linkwg/$v.$tg.$N.err \
          || { echo "$v $tg $N failed"; tail -5 gpurun_out/linkwg/$v.$tg.$N.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/linkwg/$v.$tg.$N.json')); print('$v', 'target $tg', $N, 'chain %.1f / %.1f ms' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'Z', d['Z_sha1'])"
    done
  done
done
