"""A/B of sketch kernel variants in ONE process (interleaved rounds), on the
bench's synthetic genomes.  Prints per-variant median/min kernel ms and checks
that both variants produce identical sketches.  Not part of the product."""
import os
import sys
import json
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drep_amd import _lib

N = int(os.environ.get("AB_GENOMES", 200))
L = 5_000_000
rounds = int(os.environ.get("AB_ROUNDS", 5))
variants = [int(v) for v in os.environ.get("AB_VARIANTS", "4,3").split(",")]
ctxs = {}
for v in variants:
    os.environ["DREPHIP_SKETCH_KERNEL"] = str(v)
    ctxs[v] = _lib.Context(0, 21, 1000, 42)
    ctxs[v].set_timing(True)
tile = _lib.tile_bases()
P = _lib.padded_bases([L])
tot = tile + N * P
codes = torch.zeros(tot // 16, dtype=torch.int32, device="cuda")
valid = torch.zeros(tot // 32, dtype=torch.int32, device="cuda")
ST = torch.cuda.current_stream().cuda_stream
ctxs[variants[0]].synth_device(0xD2E9, 0, N, 100, L, codes.data_ptr(), valid.data_ptr(), ST)
off = np.array([tile + i * P for i in range(N)], np.uint64)
pad = np.full(N, P, np.uint64)
nk = np.full(N, L - 20, np.uint64)
outs = {}
res = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        h = torch.zeros((N, 1000), dtype=torch.int64, device="cuda")
        n = torch.zeros(N, dtype=torch.int32, device="cuda")
        ctxs[v].sketch_device(codes.data_ptr(), valid.data_ptr(), off, pad, nk, N, h.data_ptr(), n.data_ptr(), ST)
        res[v].append(ctxs[v].kernel_ms(0)[0])
        outs[v] = h.cpu().numpy()
same = all(np.array_equal(outs[variants[0]], outs[v]) for v in variants)
kmers = N * (L - 20)
print(json.dumps({"genomes": N, "identical": same,
                  "variants": {v: {"median_ms": float(np.median(res[v])), "min_ms": float(np.min(res[v])),
                                   "Gkmer_per_s": kmers / (np.median(res[v]) / 1e3) / 1e9} for v in variants}}))
