#!/bin/bash
# Cached vs plain chain step: the linkage suite (both kernels, vs scipy), then
# tools/link_ab.py at each N in LINK_NS with DREPHIP_LINK_CACHE=1 / 0 (Z
# digest checked against scipy's committed one), launch counts from DREPHIP_DEBUG.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/linkab
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "linkage" \
    > gpurun_out/linkab/tests.log 2>&1 || { tail -30 gpurun_out/linkab/tests.log; exit 1; }
tail -1 gpurun_out/linkab/tests.log
fi
for N in ${LINK_NS:-10000}; do
  for c in 1 0; do
    DREPHIP_DEBUG=1 DREPHIP_LINK_CACHE=$c timeout -k 10 300 python tools/link_ab.py $N > gpurun_out/linkab/c$c.$N.json 2> gpurun_out/linkab/c$c.$N.err \
        || { echo "cache=$c N=$N failed"; grep -v amdgpu.ids gpurun_out/linkab/c$c.$N.err | tail -3; exit 1; }
    echo "cache=$c N=$N $(grep 'cached chain' gpurun_out/linkab/c$c.$N.err | tail -1 | cut -d: -f2)"
    python3 -c "import json; d=json.load(open('gpurun_out/linkab/c$c.$N.json')); print('   chain ms %.1f / %.1f' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'wall %.3f s' % d['wall_s_1'], 'scipy', d['Z_equals_scipy_digest'])"
  done
done
