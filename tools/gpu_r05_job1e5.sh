#!/bin/bash
# configs[3] as the sharded job on one rank over RCCL (10^5 synthetic 5 Mbp
# genomes): the stage times of drep_amd.distributed with the round-5 kernels.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05job
mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29901 \
    -m drep_amd.distributed --genomes 100000 > $O/job.json 2> $O/job.err || { tail -20 $O/job.err; exit 1; }
tail -c 3000 $O/job.json
