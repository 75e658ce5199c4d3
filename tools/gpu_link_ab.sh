#!/bin/bash
# Linkage A/B: parity tests on the default library, then the configs[3]-size
# scale test (N = 10^5, -k 100000) once per library in AB_LIBS ("lib" = the
# default drep_amd/lib, other names = drep_amd/lib_ab/<name>), linkage time printed.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "linkage or cluster_mash" --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_link.log 2>&1 || { tail -40 gpurun_out/gpu_link.log; exit 1; }
tail -1 gpurun_out/gpu_link.log
for v in ${AB_LIBS:-lib}; do
  if [ "$v" = lib ]; then L=$PWD/drep_amd/lib/libdrephip.so; else L=$PWD/drep_amd/lib_ab/$v/libdrephip.so; fi
  DREPHIP_LIB=$L DREPHIP_SCALE_OUT=gpurun_out/scale_link_$v.json timeout -k 10 600 \
     python -u -m pytest tests/test_scale.py -m gpu -x -q -s -k 100000 --timeout 580 --timeout-method thread > gpurun_out/scale_link_$v.log 2>&1 \
     || { tail -20 gpurun_out/scale_link_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/scale_link_$v.json')); print('$v', 'linkage_s %.3f' % d['linkage_s'])"
done
