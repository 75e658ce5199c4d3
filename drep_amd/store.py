"""Work-directory persistence of the Mash step at 10^4 - 10^5 genomes.

The reference stores the primary-clustering results as
  * ``data_tables/Mdb.csv`` -- the long-form Mdb, N^2 rows
    (``WorkDirectory.store_db``, drep/WorkDirectory.py:183-210; read back with
    float32 / category dtypes at 212-239), and
  * ``data/Clustering_files/primary_linkage.pickle`` -- three pickles in a row,
    [linkage, linkage_db, arguments] (``store_special('primary_linkage')``,
    WorkDirectory.py:306-313; read by ``import_clusters``, 118-134, into
    ``{'linkage', 'db', 'arguments'}``, which d_analyze.py:121-124 uses).

At 10^5 genomes the long-form Mdb is 10^10 rows and ``linkage_db`` (the
pivot) an 80 GB frame, so neither can exist.  Here the canonical form is the
condensed all-pairs result -- the integers every Mdb value is a pure function
of -- under ``data/MASH_files/condensed/``:

  common.npy   uint16 [N(N-1)/2]  shared hashes of pair (i, j), i < j, scipy
                                  squareform order
  denom.npy    uint16 [N(N-1)/2]  Mash's denominator (absent when every
                                  sketch is full: then it is s everywhere)
  nhash.npy    uint32 [N]         hashes per sketch
  length.npy   uint64 [N]         genome lengths (Mash's p-value input)
  names.txt / locations.txt       genome basenames / paths, one per line
  meta.json                       k, s, seed, N, layout

``mdb_from_condensed`` (d_cluster.py) rebuilds the exact long-form Mdb from
it when N is small, and ``primary_linkage.pickle`` is written in the
reference's own format with ``linkage_db = None`` when the pivot would not
fit (d_analyze reads only the linkage and the arguments).
"""
from __future__ import annotations

import json
import os
import pickle
from typing import Any, Dict, Optional

import numpy as np

from .d_cluster import MASH_K, MASH_SEED, CondensedMash

CONDENSED_SUBDIR = os.path.join("MASH_files", "condensed")
PRIMARY_LINKAGE = os.path.join("Clustering_files", "primary_linkage.pickle")


def condensed_dir(data_folder: str) -> str:
    return os.path.join(data_folder, CONDENSED_SUBDIR)


def store_condensed(data_folder: str, cm: CondensedMash) -> str:
    """Write cm under <data_folder>/MASH_files/condensed/ (the data folder is
    WorkDirectory.get_dir('data'), as all_vs_all_MASH receives it)."""
    d = condensed_dir(data_folder)
    os.makedirs(d, exist_ok=True)
    N = len(cm.names)
    if len(cm.common) != N * (N - 1) // 2:
        raise ValueError("common has %d pairs, expected N(N-1)/2 = %d" % (len(cm.common), N * (N - 1) // 2))
    np.save(os.path.join(d, "common.npy"), np.ascontiguousarray(cm.common, dtype=np.uint16))
    full = cm.denom is None or bool((np.asarray(cm.denom) == cm.s).all())
    dpath = os.path.join(d, "denom.npy")
    if full:
        if os.path.exists(dpath):
            os.remove(dpath)
    else:
        np.save(dpath, np.ascontiguousarray(cm.denom, dtype=np.uint16))
    np.save(os.path.join(d, "nhash.npy"), np.ascontiguousarray(cm.nhash, dtype=np.uint32))
    np.save(os.path.join(d, "length.npy"), np.ascontiguousarray(cm.length, dtype=np.uint64))
    for fname, items in (("names.txt", cm.names), ("locations.txt", cm.locations)):
        with open(os.path.join(d, fname), "w") as fh:
            for x in items:
                if "\n" in x:
                    raise ValueError("genome names/locations cannot contain newlines: %r" % x)
                fh.write(x + "\n")
    with open(os.path.join(d, "meta.json"), "w") as fh:
        json.dump({"k": MASH_K, "s": int(cm.s), "seed": MASH_SEED, "N": N, "denom_stored": not full,
                   "layout": "condensed upper triangle, index(i, j) = i*N - i*(i+1)/2 + (j - i - 1), i < j"},
                  fh, indent=1)
    return d


def load_condensed(data_folder: str, mmap: bool = True) -> CondensedMash:
    """Read what store_condensed wrote (memory-mapped by default: 10 GB of
    counts at 10^5 genomes need not be read whole)."""
    d = condensed_dir(data_folder)
    meta = json.load(open(os.path.join(d, "meta.json")))
    mode = "r" if mmap else None
    common = np.load(os.path.join(d, "common.npy"), mmap_mode=mode, allow_pickle=False)
    if meta.get("denom_stored"):
        denom = np.load(os.path.join(d, "denom.npy"), mmap_mode=mode, allow_pickle=False)
    else:
        # every sketch full: denominator s for every pair, as a zero-stride
        # read-only view (np.full would be a 10 GB host array at N = 10^5)
        denom = np.broadcast_to(np.uint16(meta["s"]), common.shape)
    names = open(os.path.join(d, "names.txt")).read().split("\n")[:meta["N"]]
    locs = open(os.path.join(d, "locations.txt")).read().split("\n")[:meta["N"]]
    return CondensedMash(names, locs, common, denom,
                         np.load(os.path.join(d, "nhash.npy"), allow_pickle=False),
                         np.load(os.path.join(d, "length.npy"), allow_pickle=False), int(meta["s"]))


def store_primary_linkage(data_folder: str, linkage: np.ndarray, linkage_db: Any,
                          arguments: Dict[str, Any]) -> str:
    """<data_folder>/Clustering_files/primary_linkage.pickle in the reference's
    format (three protocol-4 pickles: linkage, linkage_db, arguments;
    WorkDirectory.py:306-313).  linkage_db may be None (no pivot at scale)."""
    path = os.path.join(data_folder, PRIMARY_LINKAGE)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as fh:
        pickle.dump(np.asarray(linkage), fh, protocol=4)
        pickle.dump(linkage_db, fh, protocol=4)
        pickle.dump(dict(arguments), fh, protocol=4)
    return path


def load_primary_linkage(data_folder: str) -> Optional[Dict[str, Any]]:
    """The dict WorkDirectory.import_clusters builds for primary_linkage
    (WorkDirectory.py:126-132) -- for files this package wrote."""
    path = os.path.join(data_folder, PRIMARY_LINKAGE)
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        linkage = pickle.load(fh)
        db = pickle.load(fh)
        args = pickle.load(fh)
    return {"linkage": linkage, "db": db, "arguments": args}
