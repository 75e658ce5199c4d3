#!/bin/bash
# The matrix compaction of the linkage chain: the linkage suite (every method,
# compactions at many chain states), then the chain at 25000 / 50000 / 10^5
# (10^5: Z's digest must equal scipy's), compaction on and off.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py -k "linkage" > $O/test_linkage.txt 2>&1 \
    || { tail -30 $O/test_linkage.txt; exit 1; }
tail -2 $O/test_linkage.txt
for N in 100000 50000 25000; do
  for C in 1 0; do
    DREPHIP_LINK_COMPACT=$C DREPHIP_DEBUG=1 timeout -k 10 400 python -u tools/link_ab.py $N > $O/link_${N}_c$C.json 2> $O/link_${N}_c$C.err || { tail -5 $O/link_${N}_c$C.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/link_${N}_c$C.json'))
print('n=$N compact $C: chain %.1f ms (first call %.1f), launches %d (%.4f per merge), %.2f us per launch, Z==scipy %s' % (d['chain_kernel_ms_1'], d['chain_kernel_ms_0'], d['launches_1'], d['launches_per_merge'], 1e3*d['chain_kernel_ms_1']/d['launches_1'], d['Z_equals_scipy_digest']))" | tee -a $O/summary.txt
    grep "compactions" $O/link_${N}_c$C.err | tail -1 >> $O/summary.txt
  done
done
