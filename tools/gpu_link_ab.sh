#!/bin/bash
# Same-box chain A/B: the linkage suite vs scipy, then tools/link_ab.py at each
# N in LINK_NS for each variant in VARIANTS (interleaved), Z digest checked.
# A variant is "default", a lib_ab name, or "env:NAME=VAL,NAME=VAL" (default
# library with those variables).  PHASES=1 adds the phase-stamped build.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${OUT_DIR:-linkab}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "linkage" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log | tee -a $O/summary.txt
fi
for N in ${LINK_NS:-10000 100000}; do
  i=0
  for V in ${VARIANTS:-default}; do
    i=$((i+1))
    ENVS=""
    case $V in
      default) LIBV="" ;;
      env:*) LIBV=""; ENVS=$(echo ${V#env:} | tr ',' ' ') ;;
      *) LIBV=drep_amd/lib_ab/$V/libdrephip.so ;;
    esac
    env ${LIBV:+DREPHIP_LIB=$LIBV} $ENVS timeout -k 10 300 python tools/link_ab.py $N > $O/$N.$i.json 2> $O/$N.$i.err \
        || { echo "N=$N $V failed"; grep -v amdgpu.ids $O/$N.$i.err | tail -5; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$N.$i.json')); print('N=$N $V chain ms %.1f / %.1f' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'launches %d (%.4f/merge)' % (d['launches_1'], d['launches_per_merge']), 'scipy', d['Z_equals_scipy_digest'])" | tee -a $O/summary.txt
  done
  if [ "${PHASES:-0}" = 1 ]; then
    DREPHIP_LIB=drep_amd/lib_ab/phases/libdrephip.so timeout -k 10 300 python tools/link_ab.py $N > $O/$N.phases.json 2> $O/$N.phases.err \
        || { echo "phases N=$N failed"; tail -5 $O/$N.phases.err; exit 1; }
    echo "N=$N phases:" >> $O/summary.txt; grep "phase" $O/$N.phases.err | sort -u >> $O/summary.txt
  fi
done
