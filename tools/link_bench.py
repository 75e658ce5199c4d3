"""Primary-clustering linkage: GPU (drephip_linkage) vs scipy on the host, on
Mash-like condensed distances (families of related genomes, 1.0 between
families).  Not part of the product.  usage: python tools/link_bench.py N [method] [scipy 0/1]"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drep_amd import _lib

n = int(sys.argv[1]); method = sys.argv[2] if len(sys.argv) > 2 else "average"
run_scipy = len(sys.argv) <= 3 or sys.argv[3] == "1"
rng = np.random.default_rng(0)
fam = rng.integers(0, max(1, n // 100), n)
iu = np.triu_indices(n, 1)
same = fam[iu[0]] == fam[iu[1]]
y = np.ones(len(iu[0]))
y[same] = np.round(rng.random(same.sum()) * 0.2, 4)        # quantised like Mash distances
del iu, same
out = {"n": n, "method": method}
with _lib.Context(0, 21, 1000, 42) as ctx:
    ctx.set_timing(True)
    t0 = time.perf_counter(); Zg = ctx.linkage(y, method); out["gpu_s"] = time.perf_counter() - t0
    out["gpu_kernel_ms"] = ctx.kernel_ms(2)[0]
if run_scipy:
    import scipy.cluster.hierarchy as sch
    t0 = time.perf_counter(); Zs = sch.linkage(y, method=method); out["scipy_s"] = time.perf_counter() - t0
    out["identical"] = bool(np.array_equal(Zg, Zs))
print(json.dumps(out))
