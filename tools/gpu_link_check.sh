#!/bin/bash
# Linkage on the box: the GPU linkage suite against scipy, then
# tools/link_ab.py at each N in LINK_NS (chain timing; Z's digest checked
# against scipy's committed one).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/linkab
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "linkage" \
    > gpurun_out/linkab/tests.log 2>&1 || { tail -30 gpurun_out/linkab/tests.log; exit 1; }
tail -1 gpurun_out/linkab/tests.log
fi
for N in ${LINK_NS:-10000}; do
  timeout -k 10 300 python tools/link_ab.py $N > gpurun_out/linkab/$N.json 2> gpurun_out/linkab/$N.err \
      || { echo "N=$N failed"; grep -v amdgpu.ids gpurun_out/linkab/$N.err | tail -3; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/linkab/$N.json')); print('N=$N chain ms %.1f / %.1f' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'wall %.3f s' % d['wall_s_1'], 'scipy', d['Z_equals_scipy_digest'])"
done
