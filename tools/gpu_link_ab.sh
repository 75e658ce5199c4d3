#!/bin/bash
# Linkage A/B: tools/link_ab.py (synthetic configs workload, average linkage
# from the device counts, two calls) once per library in AB_LIBS (names under
# drep_amd/lib_ab/, "lib" = drep_amd/lib) and N in LINK_NS, interleaved.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/linkab
for N in ${LINK_NS:-10000 100000}; do
  for rep in 1 2; do
    for v in ${AB_LIBS:-lib}; do
      if [ "$v" = lib ]; then L=$PWD/drep_amd/lib/libdrephip.so; else L=$PWD/drep_amd/lib_ab/$v/libdrephip.so; fi
      TO=0; case "$v" in *nocol*|*timing*) TO=1;; esac
      LINK_AB_TIMING_ONLY=$TO DREPHIP_LIB=$L timeout -k 10 300 python tools/link_ab.py $N > gpurun_out/linkab/$v.$N.$rep.json 2> gpurun_out/linkab/$v.$N.$rep.err \
          || { echo "$v $N failed"; tail -5 gpurun_out/linkab/$v.$N.$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/linkab/$v.$N.$rep.json')); print('$v', $N, $rep, 'chain %.1f ms / %.1f ms' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'wall %.3f / %.3f s' % (d['wall_s_0'], d['wall_s_1']), 'alloc %.3f s' % d['phases_0']['alloc_s'], 'Z', d['Z_sha1'][:12], 'scipy' if d['Z_equals_scipy_digest'] else d['Z_equals_scipy_digest'])"
    done
  done
done
