"""All-pairs kernel timing at bench-like N on synthetic family sketches (made on
the GPU with the product sketch path), plus a bit-exact spot check of a pair
sample against the oracle.  Not part of the product."""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drep_amd import _lib
import oracle
N = int(os.environ.get("AP_N", 4000)); L = int(os.environ.get("AP_L", 2_000_000)); s = int(os.environ.get("AP_S", 1000))
PATHS = {"auto": 0, "table": 1, "band": 2, "merge": 3}
path = os.environ.get("AP_PATH", "auto")
ITERS = int(os.environ.get("AP_ITERS", 4))
ctx = _lib.Context(0, 21, s, 42); ctx.set_timing(True)
ctx.set_allpairs_path(PATHS[path], int(os.environ.get("AP_CAP", 1024)))
ST = torch.cuda.current_stream().cuda_stream
tile = _lib.tile_bases(); P = _lib.padded_bases([L]); tot = tile + N * P
codes = torch.zeros(tot // 16, dtype=torch.int32, device="cuda")
valid = torch.zeros(tot // 32, dtype=torch.int32, device="cuda")
ctx.synth_device(7, 0, N, int(os.environ.get("AP_FAM", 100)), L, codes.data_ptr(), valid.data_ptr(), ST)
h = torch.full((N, s), -1, dtype=torch.int64, device="cuda"); n = torch.zeros(N, dtype=torch.int32, device="cuda")
off = np.array([tile + i * P for i in range(N)], np.uint64)
ctx.sketch_device(codes.data_ptr(), valid.data_ptr(), off, np.full(N, P, np.uint64), np.full(N, L - 20, np.uint64), N, h.data_ptr(), n.data_ptr(), ST)
del codes, valid
npairs = N * (N - 1) // 2
out = torch.zeros(npairs, dtype=torch.int16, device="cuda")
ts = []
for it in range(ITERS):
    ctx.allpairs_device(h.data_ptr(), n.data_ptr(), N, 0, N, out.data_ptr(), None, ST)
    ts.append(ctx.kernel_ms(2)[0])
c = out.cpu().numpy().view(np.uint16)
H = h.cpu().numpy().view(np.uint64); NH = n.cpu().numpy().view(np.uint32)
rng = np.random.default_rng(0); idx = rng.integers(0, npairs, int(os.environ.get("AP_SAMPLE", 200000)))
# invert condensed index
i = np.floor(((2 * N - 1) - np.sqrt((2 * N - 1) ** 2 - 8 * idx.astype(np.float64))) / 2).astype(np.int64)
i = np.where(i * N - i * (i + 1) // 2 > idx, i - 1, i)
i = np.where((i + 1) * N - (i + 1) * (i + 2) // 2 <= idx, i + 1, i)
j = idx - (i * N - i * (i + 1) // 2) + i + 1
want = oracle.dist_pairs_list(H, NH, s, i.astype(np.uint32), j.astype(np.uint32), threads=16)
print(json.dumps({"N": N, "s": s, "L": L, "path": path, "pairs": npairs, "allpairs_ms": ts, "pairs_per_s": npairs / (min(ts) / 1e3),
                  "sample_pairs_exact": bool(np.array_equal(c[idx], want)), "common_max": int(c.max()),
                  "build_ms": ctx.kernel_ms(3)[0]}))
