"""Linkage timing on the configs' synthetic workload (not part of the product):
N synthetic 5 Mbp genomes sketched and all-pairs'ed on the GPU (as
tests/test_scale.py, no checks), then average linkage from the device counts
twice -- the first call allocates the n x n matrix, the second reuses it --
with the phase split (drephip_last_linkage_stats) and a digest of Z so runs of
different libraries (DREPHIP_LIB) can be compared.  For average linkage at a
size whose scipy digest is committed (tests/golden/scale_linkage_sha1.json:
scipy's own Z of the same counts) any other digest fails the run (exit 1),
except with LINK_AB_TIMING_ONLY=1 (timing-only builds that skip work).
usage: python tools/link_ab.py N [method]"""
import hashlib, json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drep_amd import _lib
from drep_amd.d_cluster import linkage_tables

N = int(sys.argv[1]); method = sys.argv[2] if len(sys.argv) > 2 else "average"
L, s, fam, seed = 5_000_000, 1000, 100, 0xD2E9
dev = torch.device("cuda", 0)
ctx = _lib.Context(0, 21, s, 42)
st = torch.cuda.current_stream(dev).cuda_stream
CH = min(N, 10000)
tile = _lib.tile_bases(); P = _lib.padded_bases([L])
codes = torch.zeros((tile + CH * P) // 16, dtype=torch.int32, device=dev)
valid = torch.zeros((tile + CH * P) // 32, dtype=torch.int32, device=dev)
hh = torch.full((N, s), -1, dtype=torch.int64, device=dev); nn = torch.zeros(N, dtype=torch.int32, device=dev)
for g0 in range(0, N, CH):
    n = min(CH, N - g0)
    ctx.synth_device(seed, g0, n, fam, L, codes.data_ptr(), valid.data_ptr(), st)
    ctx.sketch_device(codes.data_ptr(), valid.data_ptr(), np.array([tile + i * P for i in range(n)], np.uint64),
                      np.full(n, P, np.uint64), np.full(n, L - 20, np.uint64), n, hh[g0].data_ptr(), nn[g0:].data_ptr(), st)
del codes, valid
torch.cuda.empty_cache()
d = torch.zeros(N * (N - 1) // 2, dtype=torch.int16, device=dev)
ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, 0, N, d.data_ptr(), None, st)
torch.cuda.synchronize()
del hh, nn
lut, off = linkage_tables(np.array([s]), s)
perm = np.arange(N, dtype=np.uint32)
out = {"N": N, "method": method, "lib": os.environ.get("DREPHIP_LIB", "default")}
ctx.set_timing(True, kernels=[2, 3])
for rep in range(2):
    t0 = time.perf_counter()
    Z = ctx.linkage_counts_device(d.data_ptr(), None, N, perm, lut, off, method)
    out["wall_s_%d" % rep] = time.perf_counter() - t0
    out["phases_%d" % rep] = ctx.linkage_stats()
    out["chain_kernel_ms_%d" % rep] = ctx.kernel_ms(2)[0]
    out["launches_%d" % rep] = ctx.linkage_launches()
out["launches_per_merge"] = out["launches_1"] / (N - 1)
out["spec"] = os.environ.get("DREPHIP_LINK_SPEC", "default")
out["Z_sha1"] = hashlib.sha1(np.ascontiguousarray(Z, dtype="<f8").tobytes()).hexdigest()
golden = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                     "scale_linkage_sha1.json"))).get(str(N)) if method == "average" else None
out["Z_equals_scipy_digest"] = None if golden is None else out["Z_sha1"] == golden
print(json.dumps(out))
if golden is not None and out["Z_sha1"] != golden and os.environ.get("LINK_AB_TIMING_ONLY") != "1":
    sys.exit("Z digest %s != scipy's %s" % (out["Z_sha1"], golden))
