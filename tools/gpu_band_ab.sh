#!/bin/bash
# A/B of libdrephip builds on the band kernel (s = 10^4, N = 2000; tools/ap_bench.py), interleaved.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/bab
for rep in 1 2; do
  for v in ${AB_LIBS}; do
    DREPHIP_LIB=$PWD/drep_amd/lib_ab/$v/libdrephip.so AP_N=2000 AP_S=10000 AP_L=5000000 AP_ITERS=3 AP_SAMPLE=20000 timeout -k 10 200 python tools/ap_bench.py \
        > gpurun_out/bab/$v.$rep.json 2> gpurun_out/bab/$v.$rep.err || { echo "$v failed"; tail -5 gpurun_out/bab/$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/bab/$v.$rep.json')); print('$v', $rep, 'min %.3f ms' % min(d['allpairs_ms']), '%.3g pairs/s' % d['pairs_per_s'], 'exact', d['sample_pairs_exact'])"
  done
done
