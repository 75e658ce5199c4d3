"""The adverse-workgroup-order linkage check of
tests/test_gpu.py::test_linkage_adverse_workgroup_order as a script, for
other library builds (DREPHIP_LIB): prints {build, cases[{n, method, wg, equal}]}.
Run with DREPHIP_LINK_BATCH=32 DREPHIP_LINK_POLL=1 DREPHIP_LINK_COMPACT_MIN=100."""

import json, os, sys
import numpy as np
import scipy.cluster.hierarchy as sch
sys.path.insert(0, os.getcwd())
from drep_amd import _lib
out = {"build": _lib.build_id(), "cases": []}
rng = np.random.default_rng(17)
for n, fams in ((300, 12), (3000, 60)):
    fam = rng.integers(0, fams, n)
    iu = np.triu_indices(n, 1)
    y = np.where(fam[iu[0]] == fam[iu[1]], np.round(rng.random(len(iu[0])) * 0.2, 3), 1.0)
    for method in ("single", "complete", "average", "weighted"):
        Zs = sch.linkage(y, method=method)
        for wg in ("64", "256"):
            if method == "single" and wg == "64":
                continue
            os.environ["DREPHIP_LINK_WG"] = wg
            with _lib.Context(0, 21, 1000, 42) as ctx:
                ctx.set_linkage_path(ctx.LINK_DENSE)
                Z = ctx.linkage(y, method)
            out["cases"].append({"n": n, "method": method, "wg": wg, "equal": bool(np.array_equal(Z, Zs))})
print(json.dumps(out))
