"""Which resource binds the sketch hash kernel (k_sketch_hash21)?  Same-box
timing of the hash kernel (HIP events, first threshold round only) at
configs[1] (1000 synthetic 5 Mbp genomes) for the libraries given in
DREPHIP_LIB, under the ablation build's index mask (EXTRA=-DDREPHIP_SK_ABLATE=1,
tools/build_ab.sh): DREPHIP_SK_KMASK=0x3FF (real lookups) against 0 (every lane
reads table entry 0: LDS broadcast, no bank conflicts, the same instructions).
Not product code; the outputs of the masked runs are not sketches.
usage: DREPHIP_LIB=... [DREPHIP_SK_KMASK=...] DREPHIP_SK_ONE_ROUND=1 python tools/sketch_ablate.py [reps]"""
import json
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drep_amd import _lib

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
N, L, s, fam, seed = 1000, 5_000_000, 1000, 100, 0xD2E9
dev = torch.device("cuda", 0)
ctx = _lib.Context(0, 21, s, 42)
st = torch.cuda.current_stream(dev).cuda_stream
tile = _lib.tile_bases(); P = _lib.padded_bases([L])
codes = torch.zeros((tile + N * P) // 16, dtype=torch.int32, device=dev)
valid = torch.zeros((tile + N * P) // 32, dtype=torch.int32, device=dev)
ctx.synth_device(seed, 0, N, fam, L, codes.data_ptr(), valid.data_ptr(), st)
hh = torch.full((N, s), -1, dtype=torch.int64, device=dev); nn = torch.zeros(N, dtype=torch.int32, device=dev)
off = np.array([tile + i * P for i in range(N)], np.uint64)
ctx.set_timing(True, kernels=[0])
ms = []
for r in range(reps + 2):
    ctx.sketch_device(codes.data_ptr(), valid.data_ptr(), off, np.full(N, P, np.uint64), np.full(N, L - 20, np.uint64),
                      N, hh.data_ptr(), nn.data_ptr(), st)
    torch.cuda.synchronize()
    if r >= 2:
        ms.append(ctx.kernel_ms(0)[0])
out = {"lib": os.environ.get("DREPHIP_LIB", "default"), "kmask": os.environ.get("DREPHIP_SK_KMASK", "none"),
       "hash_ms_median": float(np.median(ms)), "hash_ms_min": float(np.min(ms)), "reps": reps}
print(json.dumps(out), flush=True)
