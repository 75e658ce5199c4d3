"""Compare the stored results of two drep_amd.distributed runs (--out folders):
condensed counts, nhash, names, linkage Z and primary Cdb must be equal.
usage: python tools/compare_jobs.py <out_a> <out_b>  (prints one JSON line, exit 1 on a difference)"""
import json
import os
import sys
import numpy as np
import pandas as pd
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drep_amd.store import load_condensed, load_primary_linkage

a, b = sys.argv[1], sys.argv[2]
ca, cb = load_condensed(a, mmap=False), load_condensed(b, mmap=False)
la, lb = load_primary_linkage(a), load_primary_linkage(b)
da, db = pd.read_csv(os.path.join(a, "primary_Cdb.csv")), pd.read_csv(os.path.join(b, "primary_Cdb.csv"))
res = {"a": a, "b": b, "genomes": len(ca.names), "pairs": int(len(ca.common)),
       "names_equal": ca.names == cb.names,
       "counts_equal": bool(np.array_equal(ca.common, cb.common)),
       "nhash_equal": bool(np.array_equal(ca.nhash, cb.nhash)),
       "Z_equal": bool(np.array_equal(la["linkage"], lb["linkage"])),
       "Cdb_equal": bool(da.equals(db)),
       "primary_clusters": int(da["primary_cluster"].nunique()),
       "pairs_sharing_a_hash": int((ca.common > 0).sum())}
res["all_equal"] = all(res[k] for k in ("names_equal", "counts_equal", "nhash_equal", "Z_equal", "Cdb_equal"))
print(json.dumps(res))
sys.exit(0 if res["all_equal"] else 1)
