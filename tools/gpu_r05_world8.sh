#!/bin/bash
# World-8 rehearsal on one MI355X before the driver's 8-GPU run: 8 ranks share
# the GPU over gloo (RCCL needs a GPU per rank).
#  1. bench.py --gpus 8 at configs[1] with --verify 1 (every rank re-sketches
#     all genomes and recomputes the whole triangle, checks its gathered
#     sketches and its segment);
#  2. drep_amd.distributed at configs[2] size (10^4 synthetic 5 Mbp genomes,
#     1250 per rank), the screen forced on in every rank and the root's
#     condensed vector starting poisoned, against the same job on 1 rank:
#     stored counts, Z and Cdb equal (tools/compare_jobs.py).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05w8
mkdir -p $O
export MASTER_ADDR=127.0.0.1
DREPHIP_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 8 --steps 5 --warmup 2 --verify 1 --cpu-baseline 0 \
    > $O/bench_gpus8.json 2> $O/bench_gpus8.err || { tail -20 $O/bench_gpus8.err; exit 1; }
tail -c 1500 $O/bench_gpus8.json
python3 -c "import json; d=json.loads(open('$O/bench_gpus8.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('n_gpus','ranks_seen','backend','verified_against_single_gpu','verified','ms_per_step')})"
for W in 1 8; do
  DREPHIP_DIST_BACKEND=gloo DREPHIP_SEGMENT_POISON=1 DREPHIP_AP_SCREEN=1 timeout -k 10 500 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29800 + W)) \
    -m drep_amd.distributed --genomes 10000 --out /tmp/r05w8_job_w$W > $O/job_w$W.json 2> $O/job_w$W.err \
    || { echo "job W=$W failed"; tail -20 $O/job_w$W.err; exit 1; }
  tail -1 $O/job_w$W.json
done
python tools/compare_jobs.py /tmp/r05w8_job_w1 /tmp/r05w8_job_w8 | tee $O/compare.json
