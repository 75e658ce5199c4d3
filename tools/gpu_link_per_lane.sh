#!/bin/bash
# Linkage step-kernel grid density A/B (DREPHIP_LINK_PER_LANE: entries per lane
# of a step, i.e. n / (256 * per) workgroups; "auto" = the library's choice)
# on tools/link_ab.py, interleaved.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/linkpl
for N in ${LINK_NS:-100000}; do
  for rep in 1 2; do
    for per in ${PERS:-2 4 8 16}; do
      if [ "$per" = auto ]; then unset DREPHIP_LINK_PER_LANE; else export DREPHIP_LINK_PER_LANE=$per; fi
      DREPHIP_LINK_PATH=dense timeout -k 10 300 python tools/link_ab.py $N > gpurun_out/linkpl/$per.$N.$rep.json 2> gpurun_out/linkpl/$per.$N.$rep.err \
          || { echo "$per $N failed"; tail -5 gpurun_out/linkpl/$per.$N.$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/linkpl/$per.$N.$rep.json')); print('per', '$per', $N, $rep, 'chain %.1f ms / %.1f ms' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'wall %.3f / %.3f s' % (d['wall_s_0'], d['wall_s_1']), 'Z', d['Z_sha1'])"
    done
  done
done
