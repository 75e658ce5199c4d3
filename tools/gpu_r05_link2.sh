#!/bin/bash
# Round-5 linkage pass 2: suite vs scipy, then at 10^4 and 10^5 the product
# chain (scalar decision, write-through column stores) against lib_ab variants:
# prevdec (the previous decision code, same stores), col1 (plain column
# stores), row3 (write-through row stores); then the phase-stamped build.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05link2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "linkage" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log | tee -a $O/summary.txt
for N in 10000 100000; do
  for LIB in default prevdec col1 row3 default; do
    if [ $LIB = default ]; then unset DREPHIP_LIB; else export DREPHIP_LIB=drep_amd/lib_ab/$LIB/libdrephip.so; fi
    timeout -k 10 300 python tools/link_ab.py $N > $O/$N.$LIB.json 2> $O/$N.$LIB.err \
        || { echo "N=$N $LIB failed"; grep -v amdgpu.ids $O/$N.$LIB.err | tail -5; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$N.$LIB.json')); print('N=$N $LIB chain ms %.1f / %.1f' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'launches %d (%.4f/merge)' % (d['launches_1'], d['launches_per_merge']), 'scipy', d['Z_equals_scipy_digest'])" | tee -a $O/summary.txt
  done
  unset DREPHIP_LIB
  DREPHIP_LIB=drep_amd/lib_ab/phases/libdrephip.so timeout -k 10 300 python tools/link_ab.py $N > $O/$N.phases.json 2> $O/$N.phases.err \
      || { echo "phases N=$N failed"; tail -5 $O/$N.phases.err; exit 1; }
  echo "N=$N phases:" >> $O/summary.txt; grep "phase" $O/$N.phases.err | sort -u >> $O/summary.txt
done
cat $O/summary.txt
