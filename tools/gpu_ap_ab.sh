#!/bin/bash
# A/B of libdrephip builds on the all-pairs kernel (tools/ap_bench.py) at
# several N, interleaved.  AB_LIBS names drep_amd/lib_ab/<name>/libdrephip.so.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/apab
for N in ${AP_NS:-1000 6000 20000}; do
  for rep in 1 2; do
    for v in ${AB_LIBS}; do
      DREPHIP_LIB=$PWD/drep_amd/lib_ab/$v/libdrephip.so AP_N=$N AP_ITERS=5 AP_SAMPLE=20000 timeout -k 10 120 python tools/ap_bench.py \
          > gpurun_out/apab/$v.$N.$rep.json 2> gpurun_out/apab/$v.$N.$rep.err || { echo "$v $N failed"; tail -5 gpurun_out/apab/$v.$N.$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/apab/$v.$N.$rep.json')); print('$v', $N, $rep, 'min %.4f ms' % min(d['allpairs_ms']), '%.3g pairs/s' % d['pairs_per_s'], 'exact', d['sample_pairs_exact'])"
    done
  done
done
