#!/bin/bash
# Round-5 linkage pass: the GPU linkage suite against scipy, then the chain at
# 10^4 and 10^5 (configs workload) with the round-4 protocol (DREPHIP_LINK_SPEC=1)
# and the round-5 one (default, known-merge speculation), interleaved; Z's digest
# checked against scipy's committed one in every run.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05link
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "linkage" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
for N in ${LINK_NS:-10000 100000}; do
  for SP in ${LINK_SPECS:-2 1 2}; do
    DREPHIP_LINK_SPEC=$SP DREPHIP_DEBUG=1 timeout -k 10 400 python tools/link_ab.py $N > $O/$N.spec$SP.json 2> $O/$N.spec$SP.err \
        || { echo "N=$N spec=$SP failed"; grep -v amdgpu.ids $O/$N.spec$SP.err | tail -5; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$N.spec$SP.json')); print('N=$N spec=$SP chain ms %.1f / %.1f' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'launches %d (%.4f/merge)' % (d['launches_1'], d['launches_per_merge']), 'wall %.3f s' % d['wall_s_1'], 'scipy', d['Z_equals_scipy_digest'])" | tee -a $O/summary.txt
  done
done
# column-y store flavour at 10^5 (the merged column leaves ~10^5 dirty lines per merge launch):
# plain (product) vs write-through sc1 (lib_ab/col3) vs nontemporal (lib_ab/col2), interleaved
if [ "${COLSTORE_AB:-1}" = 1 ]; then
for LIB in default col3 col2 default col3; do
  if [ $LIB = default ]; then unset DREPHIP_LIB; else export DREPHIP_LIB=drep_amd/lib_ab/$LIB/libdrephip.so; fi
  timeout -k 10 400 python tools/link_ab.py 100000 > $O/col_$LIB.json 2> $O/col_$LIB.err \
      || { echo "colstore $LIB failed"; grep -v amdgpu.ids $O/col_$LIB.err | tail -5; exit 1; }
  python3 -c "import json; d=json.load(open('$O/col_$LIB.json')); print('colstore $LIB N=100000 chain ms %.1f / %.1f' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'launches %d' % d['launches_1'], 'scipy', d['Z_equals_scipy_digest'])" | tee -a $O/summary.txt
done
unset DREPHIP_LIB
fi
