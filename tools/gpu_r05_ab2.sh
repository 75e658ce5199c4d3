#!/bin/bash
# Distance-matrix build with batched lookups (default) vs the committed build (bf):
# the linkage suite, then link_ab at 10^4 and 10^5 (matrix_s and Z digest).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05ab2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "linkage or dist_matrix or cluster" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log | tee -a $O/summary.txt
for N in 10000 100000; do
  for V in bf default bf default; do
    LIBV=""; [ $V != default ] && LIBV=drep_amd/lib_ab/$V/libdrephip.so
    env ${LIBV:+DREPHIP_LIB=$LIBV} timeout -k 10 300 python tools/link_ab.py $N > $O/$N.$V.json 2> $O/$N.$V.err || { tail -5 $O/$N.$V.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/$N.$V.json'))
print('N=$N $V matrix %.1f / %.1f ms, chain %.1f ms, Z %s scipy %s' % (1e3*d['phases_0']['matrix_s'], 1e3*d['phases_1']['matrix_s'], d['chain_kernel_ms_1'], d['Z_sha1'][:12], d['Z_equals_scipy_digest']))" | tee -a $O/summary.txt
  done
done
