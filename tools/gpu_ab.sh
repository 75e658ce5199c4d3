#!/bin/bash
# A/B of libdrephip builds (drep_amd/lib_ab/<name>/libdrephip.so) on the default
# bench: sketch hash kernel time and step time, interleaved runs.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${AB_LIBS}; do
    DREPHIP_LIB=$PWD/drep_amd/lib_ab/$v/libdrephip.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 ${BENCH_ARGS} \
        > gpurun_out/ab/$v.$rep.json 2> gpurun_out/ab/$v.$rep.err || { echo "$v failed"; tail -5 gpurun_out/ab/$v.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.$rep.json')); k=d['kernels_rank0']; print('$v', $rep, 'step %.3f ms' % d['ms_per_step'], 'hash %.3f ms' % k['sketch_hash_ms_avg'], 'allpairs %.3f' % k['allpairs_ms_avg'], 'verified', d.get('verified'))"
  done
done
