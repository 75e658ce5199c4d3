#!/bin/bash
# The sharded bench path (torchrun, 2 and 3 ranks) rehearsed on ONE GPU over
# gloo, pipelined and one-step host loops, with --verify (each rank's gathered
# sketches and condensed segment checked against a single-GPU recomputation).
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export DREPHIP_DIST_BACKEND=gloo
for spec in "2 1" "3 1" "2 0"; do
  w=${spec% *}; p=${spec#* }
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
      --master-port $((29500 + w * 10 + p)) bench.py --gpus $w --genomes 201 --steps 3 --warmup 1 --verify 1 \
      --cpu-baseline 0 --pipeline $p > gpurun_out/mr_w${w}_p$p.json 2> gpurun_out/mr_w${w}_p$p.err \
      || { echo "world $w pipeline $p failed"; tail -30 gpurun_out/mr_w${w}_p$p.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/mr_w${w}_p$p.json').read().strip().splitlines()[-1]); print('world', $w, 'pipe', $p, d['ms_per_step'], d.get('verified_against_single_gpu'), d['config']['host_loop'])"
done
unset DREPHIP_DIST_BACKEND
timeout -k 10 200 python bench.py --genomes 201 --steps 3 --warmup 1 --verify 1 --cpu-baseline 0 > gpurun_out/mr_w1.json 2> gpurun_out/mr_w1.err || { echo "world 1 failed"; tail gpurun_out/mr_w1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/mr_w1.json')); print('world 1', d['ms_per_step'], d.get('verified_against_single_gpu'), d['config']['host_loop'])"
