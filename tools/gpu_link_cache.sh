#!/bin/bash
# The cache-driven chain step on the box: the linkage suite against scipy
# (both step kernels), then chain timings at 10^4 / 10^5 for
# DREPHIP_LINK_CACHE=1 and 0 with Z checked against scipy's committed digest.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/linkab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "linkage" \
    > gpurun_out/linkab/tests.log 2>&1 || { tail -30 gpurun_out/linkab/tests.log; exit 1; }
tail -3 gpurun_out/linkab/tests.log
for N in ${LINK_NS:-10000 100000}; do
  for c in 1 0; do
    DREPHIP_LINK_CACHE=$c timeout -k 10 300 python tools/link_ab.py $N > gpurun_out/linkab/cache$c.$N.json 2> gpurun_out/linkab/cache$c.$N.err \
        || { echo "cache=$c $N failed"; tail -5 gpurun_out/linkab/cache$c.$N.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/linkab/cache$c.$N.json')); print('cache=$c', $N, 'chain %.1f ms / %.1f ms' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'wall %.3f / %.3f s' % (d['wall_s_0'], d['wall_s_1']), 'Z', d['Z_sha1'][:12], 'scipy' if d['Z_equals_scipy_digest'] else d['Z_equals_scipy_digest'])"
  done
done
