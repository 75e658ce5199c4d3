"""One rank's step of the W-way sharded bench, rehearsed on one GPU (not part of
the product): the rank sketches its N/W genome shard, the full N-genome sketch
matrix stands in for the all-gather result, and the rank runs all-pairs over
its balanced row range.  Reports ms per step and the per-kernel times, so the
fixed per-step overheads that dominate at 8 GPUs can be measured.
    python tools/shard_step.py [N] [W] [rank] [steps]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drep_amd import _lib                                       # noqa: E402
from drep_amd.parallel import genome_shard, row_partition, segment_size   # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
W = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
L, s, fam = 5_000_000, 1000, 100
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev).cuda_stream
ctx = _lib.Context(device=0, k=21, s=s, seed=42)
tile, P = _lib.tile_bases(), _lib.padded_bases([L])

# the full sketch matrix (stands in for the all-gather result)
codes = torch.zeros((tile + N * P) // 16, dtype=torch.int32, device=dev)
valid = torch.zeros((tile + N * P) // 32, dtype=torch.int32, device=dev)
ctx.synth_device(0, 0, N, fam, L, codes.data_ptr(), valid.data_ptr(), stream)
full_h = torch.full((N, s), -1, dtype=torch.int64, device=dev)
full_n = torch.zeros(N, dtype=torch.int32, device=dev)
ctx.sketch_device(codes.data_ptr(), valid.data_ptr(), np.array([tile + i * P for i in range(N)], np.uint64),
                  np.full(N, P, np.uint64), np.full(N, L - 20, np.uint64), N, full_h.data_ptr(), full_n.data_ptr(),
                  stream)
del codes, valid

g0, g1, nmax = genome_shard(N, W, rank)
n = g1 - g0
codes = torch.zeros((tile + n * P) // 16, dtype=torch.int32, device=dev)
valid = torch.zeros((tile + n * P) // 32, dtype=torch.int32, device=dev)
ctx.synth_device(0, g0, n, fam, L, codes.data_ptr(), valid.data_ptr(), stream)
base_off = np.array([tile + i * P for i in range(n)], np.uint64)
padded, nk = np.full(n, P, np.uint64), np.full(n, L - 20, np.uint64)
loc_h = torch.full((nmax, s), -1, dtype=torch.int64, device=dev)
loc_n = torch.zeros(nmax, dtype=torch.int32, device=dev)
r0, r1 = row_partition(N, W)[rank]
d_common = torch.zeros(max(segment_size(N, r0, r1), 1), dtype=torch.int16, device=dev)
timing = os.environ.get("SHARD_TIMING", "1") == "1"
ctx.set_timing(timing)
kms = np.zeros(4)


defer = os.environ.get("SHARD_DEFER", "1") == "1"     # bench default: status checked after all-pairs


def step():
    (ctx.sketch_device_async if defer else ctx.sketch_device)(
        codes.data_ptr(), valid.data_ptr(), base_off, padded, nk, n, loc_h.data_ptr(), loc_n.data_ptr(), stream)
    if timing and not defer:
        for w in (0, 1):
            kms[w] += ctx.kernel_ms(w)[0]
    ctx.allpairs_device(full_h.data_ptr(), full_n.data_ptr(), N, r0, r1, d_common.data_ptr(), None, stream)
    if timing:
        for w in (2, 3):
            kms[w] += ctx.kernel_ms(w)[0]
    if defer:
        assert not ctx.sketch_wait()
        if timing:
            for w in (0, 1):
                kms[w] += ctx.kernel_ms(w)[0]


pipe = os.environ.get("SHARD_PIPE", "1") == "1"       # bench default: host one step ahead


def pipelined(k):
    for i in range(k):
        if i > 0:
            assert not ctx.sketch_wait()
        ctx.sketch_device_async(codes.data_ptr(), valid.data_ptr(), base_off, padded, nk, n, loc_h.data_ptr(),
                                loc_n.data_ptr(), stream)
        if i > 0:
            ctx.allpairs_wait()
        ctx.allpairs_device_async(full_h.data_ptr(), full_n.data_ptr(), N, r0, r1, d_common.data_ptr(), None,
                                  stream)
    assert not ctx.sketch_wait()
    ctx.allpairs_wait()


if pipe:
    ctx.set_timing(False)
    timing = False
for _ in range(3):
    step()
torch.cuda.synchronize()
kms[:] = 0
t0 = time.perf_counter()
if pipe:
    pipelined(steps)
else:
    for _ in range(steps):
        step()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / steps * 1e3
assert torch.equal(loc_h[:n], full_h[g0:g1]), "shard sketches differ from the full run"
k = kms / steps
print(json.dumps({"N": N, "W": W, "rank": rank, "genomes": n, "rows": [r0, r1], "timing_events": timing,
                  "deferred_check": defer, "pipelined": pipe,
                  "ms_per_step": ms, "sketch_hash_ms": k[0], "finalize_ms": k[1], "allpairs_ms": k[2],
                  "build_ms": k[3], "overhead_ms": ms - k.sum() if timing else None}))
