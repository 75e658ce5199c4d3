"""Same-process A/B of all-pairs kernel variants selected by an environment
variable read per call (AB_VAR, default DREPHIP_AP_R: the whole-row
kernel's rows per workgroup; round 4 also compared the band kernel's
geometries this way, profiles/r04_band_geometry_ab.json) on the configs'
workload: N synthetic 5 Mbp genomes (families of 100, the bench's generator)
sketched at s = AB_S (1000 by default; 10^4 is configs[4]) on the GPU, then every variant timed in interleaved rounds (HIP events around
the kernel) and its WHOLE triangle compared with the literal merge kernel's
(k_allpairs_merge).  Not part of the product.
usage: python tools/ap_ab.py [N] [values, e.g. 4,8] [rounds]; values "" times the library as it is"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drep_amd import _lib

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
cfgs = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4,8").split(",") if x]
VAR = os.environ.get("AB_VAR", "DREPHIP_AP_R")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
s, L, fam, seed = int(os.environ.get("AB_S", 1000)), 5_000_000, int(os.environ.get("AB_FAM", 100)), 0xD2E9
dev = torch.device("cuda", 0)
ctx = _lib.Context(0, 21, s, 42)
st = torch.cuda.current_stream(dev).cuda_stream
CH = min(N, 4000)
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
torch.cuda.synchronize(); torch.cuda.empty_cache()
npairs = N * (N - 1) // 2
ref = torch.empty(npairs, dtype=torch.int16, device=dev)
t0 = time.perf_counter()
if os.environ.get("AB_NOREF") != "1":       # AB_NOREF=1: timing only, no whole-triangle check
    ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, 0, N, ref.data_ptr(), None, st, merge=True)
torch.cuda.synchronize()
out = {"N": N, "s": s, "pairs": npairs, "merge_s": time.perf_counter() - t0, "cfg": {}}
print("reference (literal merge) done in %.2f s" % out["merge_s"], file=sys.stderr, flush=True)
ctx.set_timing(True, kernels=[2, 4])
got = torch.empty(npairs, dtype=torch.int16, device=dev)
for rd in range(rounds):
    for c in (cfgs or [-1]):
        if c >= 0:
            os.environ[VAR] = str(c)
        got.fill_(0x7FFF)
        ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, 0, N, got.data_ptr(), None, st)
        # the all-pairs kernel (with the no-shared-hash fill when screened) plus the screen itself
        ms = ctx.kernel_ms(2)[0] + (ctx.kernel_ms(4)[0] if hasattr(_lib.lib(), "drephip_last_screen_stats") else 0.0)
        bad = int((got != ref).sum().item()) if os.environ.get("AB_NOREF") != "1" else 0
        r = out["cfg"].setdefault(str(c), {"ms": [], "mismatches": 0})
        if hasattr(_lib.lib(), "drephip_last_screen_stats"):       # libraries from before round 4 have no screen
            r["screen"] = ctx.screen_stats()
            r["screen_ms"] = ctx.kernel_ms(4)[0]
            print("  stats %s=%d: %s, screen %.3f ms" % (VAR, c, r["screen"], r["screen_ms"]), file=sys.stderr,
                  flush=True)
        r["ms"].append(ms); r["mismatches"] += bad
        print("round %d %s=%d: %.3f ms, %d mismatches" % (rd, VAR, c, ms, bad), file=sys.stderr, flush=True)
for c, r in out["cfg"].items():
    r["min_ms"] = min(r["ms"]); r["pairs_per_s"] = npairs / (r["min_ms"] / 1e3)
print(json.dumps(out))
sys.exit(1 if any(r["mismatches"] for r in out["cfg"].values()) else 0)
