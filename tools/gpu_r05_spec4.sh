#!/bin/bash
# Spec 4 (speculation in every merge launch, y's own minimum in a fourth
# partial set) re-built on the final step kernel: the linkage suite with it
# (DREPHIP_LINK_SPEC=3), then the chain at 10^4 / 10^5, interleaved: bf = HEAD's
# library, default = this library at spec level 2, spec3 = this library at 3.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05spec4
mkdir -p $O
DREPHIP_LINK_SPEC=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "linkage" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log | tee -a $O/summary.txt
for N in 10000 100000; do
  for V in bf default spec3 bf default spec3; do
    LIBV=""; ENVS=""
    [ $V = bf ] && LIBV=drep_amd/lib_ab/bf/libdrephip.so
    [ $V = spec3 ] && ENVS="DREPHIP_LINK_SPEC=3"
    env ${LIBV:+DREPHIP_LIB=$LIBV} $ENVS DREPHIP_DEBUG=1 timeout -k 10 300 python tools/link_ab.py $N > $O/$N.$V.json 2> $O/$N.$V.err || { tail -5 $O/$N.$V.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/$N.$V.json'))
print('N=$N $V chain %.1f / %.1f ms, launches %d (%.4f per merge), scipy %s' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1'], d['launches_1'], d['launches_per_merge'], d['Z_equals_scipy_digest']))" | tee -a $O/summary.txt
  done
done
