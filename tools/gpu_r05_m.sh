#!/bin/bash
# The 8-rank job's invalid Z (tools/gpu_r05_world8.sh): the gathered counts of
# 1-rank and 8-rank jobs at 10^4 genomes with the light screen on and off, compared
# pair by pair; then the multi-rank GPU tests.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05m
mkdir -p $O
export MASTER_ADDR=127.0.0.1
for L in 1 0; do
  for W in 1 8; do
    DREPHIP_SCREEN_LIGHT=$L DREPHIP_DUMP_COUNTS=/tmp/cnt_l${L}_w$W.npy DREPHIP_DIST_BACKEND=gloo DREPHIP_SEGMENT_POISON=1 \
      DREPHIP_AP_SCREEN=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
      --master-addr 127.0.0.1 --master-port $((29700 + W + 10 * L)) -m drep_amd.distributed --genomes 10000 \
      --out /tmp/r05m_l${L}_w$W > $O/job_l${L}_w$W.json 2> $O/job_l${L}_w$W.err
    echo "light $L world $W rc $?" | tee -a $O/summary.txt
    grep -h "Error\|error" $O/job_l${L}_w$W.err | grep -v amdgpu.ids | head -3 >> $O/summary.txt
  done
done
python3 - <<'PY' | tee -a gpurun_out/r05m/summary.txt
import numpy as np, os
f = lambda p: np.load(p) if os.path.exists(p) else None
a = {k: f('/tmp/cnt_%s.npy' % k) for k in ('l1_w1', 'l1_w8', 'l0_w1', 'l0_w8')}
for x, y in (('l1_w1', 'l1_w8'), ('l0_w1', 'l0_w8'), ('l1_w1', 'l0_w1')):
    if a[x] is None or a[y] is None:
        print(x, y, 'missing'); continue
    d = np.nonzero(a[x] != a[y])[0]
    print(x, y, 'differ at', len(d), 'pairs', d[:10].tolist(), a[x][d[:10]].tolist(), a[y][d[:10]].tolist())
    if len(d):
        N = 10000
        i = np.searchsorted(np.array([r * N - r * (r + 1) // 2 for r in range(N)]), d[:10], side='right') - 1
        print('rows', i.tolist())
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py > $O/dist_tests.log 2>&1
tail -3 $O/dist_tests.log | tee -a $O/summary.txt
