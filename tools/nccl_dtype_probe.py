"""Which tensor dtypes torch's nccl (RCCL) process group accepts, on one GPU
(world size 1): the condensed counts are uint16, which NCCL has no type for,
so drep_amd.distributed moves them as int8 byte views."""
import os
import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for dt in (torch.int16, torch.int8, torch.int32, torch.int64):
    t = torch.ones(5, dtype=dt, device="cuda")
    try:
        dist.all_reduce(t)
        torch.cuda.synchronize()
        print(dt, "accepted")
    except Exception as e:          # noqa: BLE001 -- report the refusal
        print(dt, "refused:", str(e).splitlines()[0][:120])
dist.destroy_process_group()
