import sys, numpy as np
sys.path.insert(0, '/root/repo')
import scipy.cluster.hierarchy as sch
from drep_amd import _lib
n=257; method='average'
rng=np.random.default_rng(n*31+len(method)); m=n*(n-1)//2
vals=np.array([0.0,0.00243596,0.0157245,0.0157245,0.05,0.1,0.243761,1.0,1.0,1.0]); y=vals[rng.integers(0,len(vals),m)]
Zs=sch.linkage(y,method=method)
with _lib.Context(0,21,1000,42) as ctx:
    Z=ctx.linkage(y,method)
bad=np.argwhere(Z!=Zs)
print("ndiff", len(bad))
for r in sorted(set(bad[:,0]))[:8]:
    print(r, Z[r].tolist(), Zs[r].tolist(), (Z[r,2]-Zs[r,2]))
