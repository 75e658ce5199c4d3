"""Per-launch time of the sketch hash kernel on the bench workload (1000
synthetic 5 Mbp genomes, s = 1000), for A/B builds (DREPHIP_LIB): HIP events
around every hash launch (drephip timing index 0), averaged over the launches of
a few sketch calls.  Not part of the product.  usage: python tools/sketch_kernel_time.py [reps]"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drep_amd import _lib

N, L, s, fam, seed = 1000, 5_000_000, 1000, 100, 0xD2E9
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
ctx = _lib.Context(0, 21, s, 42)
st = torch.cuda.current_stream(dev).cuda_stream
tile = _lib.tile_bases(); P = _lib.padded_bases([L])
codes = torch.zeros((tile + N * P) // 16, dtype=torch.int32, device=dev)
valid = torch.zeros((tile + N * P) // 32, dtype=torch.int32, device=dev)
ctx.synth_device(seed, 0, N, fam, L, codes.data_ptr(), valid.data_ptr(), st)
hh = torch.zeros((N, s), dtype=torch.int64, device=dev); nn = torch.zeros(N, dtype=torch.int32, device=dev)
off = np.array([tile + i * P for i in range(N)], np.uint64)
args = (codes.data_ptr(), valid.data_ptr(), off, np.full(N, P, np.uint64), np.full(N, L - 20, np.uint64), N,
        hh.data_ptr(), nn.data_ptr(), st)
ctx.sketch_device(*args)
ctx.set_timing(True, kernels=[0])
tot, launches = 0.0, 0
for _ in range(reps):
    ctx.sketch_device(*args)
    ms, k = ctx.kernel_ms(0)
    tot += ms; launches += k
print(json.dumps({"lib": os.environ.get("DREPHIP_LIB", "default"), "hash_ms_per_launch": tot / launches,
                  "launches": launches, "calls": reps}))
