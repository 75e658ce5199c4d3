#!/bin/bash
# The screen tests after the light cells were tied to the band kernel; chain
# cost per launch against n (25000, 50000, 10^5: the case for compacting the
# matrix as clusters retire).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_screen.py > $O/test_screen.txt 2>&1 \
    || { tail -20 $O/test_screen.txt; exit 1; }
tail -2 $O/test_screen.txt
for N in 25000 50000 100000; do
  DREPHIP_DEBUG=1 timeout -k 10 400 python -u tools/link_ab.py $N > $O/link_$N.json 2> $O/link_$N.err || { tail -5 $O/link_$N.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/link_$N.json'))
print('n=$N chain %.1f ms, launches %d (%.4f per merge), %.2f us per launch, Z==scipy %s' % (d['chain_kernel_ms_1'], d['launches_1'], d['launches_per_merge'], 1e3*d['chain_kernel_ms_1']/d['launches_1'], d['Z_equals_scipy_digest']))" | tee -a $O/summary.txt
done
