"""Time the Mash branch of dRep's cluster_genomes through the drop-in.

The reference's branch (drep/d_cluster.py:168-185) is

    Mdb = all_vs_all_MASH(Bdb, data_folder, **kwargs)           # 170
    Cdb, cluster_ret = cluster_mash_database(Mdb, **kwargs)      # 177
    wd.store_special('primary_linkage', cluster_ret)             # 185

This runs exactly that with drep_amd.d_cluster's functions on N synthetic
genomes (BASELINE's generator, sketched on the GPU during setup and written as
dRep's per-genome .msh cache, MASH_files/sketches/chunk_<i>/<genome>.msh, so
the timed call reuses them as dRep does on a rerun, d_cluster.py:541-542; FASTA
ingest is measured elsewhere), with the CLI's kwargs (MASH_sketch as a string,
clusterAlg, P_ani, processors, groupSize), and the stored primary_linkage in
the reference's pickle layout (drep_amd.store).  Genome names are a shuffled
set, so Bdb order differs from the pivot's sorted order.

--reference-leg then runs the reference's own cluster_mash_database steps on
the same Mdb (the in-place dist update, pandas' pivot, squareform, scipy's
linkage, fcluster; d_cluster.py:445-459, 619-623) and checks linkage_db, Z and
Cdb against the drop-in's bit for bit.

    python tools/dropin_bench.py --genomes 10000 --reference-leg --out profiles/r06_dropin_10000.json
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def synth_sketches(N: int, L: int, family_size: int, s: int, seed: int):
    """uint64 [N, s] sketches + nhash of BASELINE's synthetic genomes (the
    bench's on-device generator and the product sketch kernel)."""
    import torch
    from drep_amd import _lib
    tile = _lib.tile_bases()
    P = _lib.padded_bases([L])
    CH = min(N, 1000)
    H = np.empty((N, s), np.uint64)
    NH = np.empty(N, np.uint32)
    with _lib.Context(0, 21, s, 42) as ctx:
        st = torch.cuda.current_stream().cuda_stream
        codes = torch.zeros((tile + CH * P) // 16, dtype=torch.int32, device="cuda")
        valid = torch.zeros((tile + CH * P) // 32, dtype=torch.int32, device="cuda")
        hh = torch.zeros((CH, s), dtype=torch.int64, device="cuda")
        nn = torch.zeros(CH, dtype=torch.int32, device="cuda")
        for a in range(0, N, CH):
            m = min(CH, N - a)
            ctx.synth_device(seed, a, m, family_size, L, codes.data_ptr(), valid.data_ptr(), st)
            ctx.sketch_device(codes.data_ptr(), valid.data_ptr(), np.array([tile + i * P for i in range(m)], np.uint64),
                              np.full(m, P, np.uint64), np.full(m, L - 20, np.uint64), m, hh.data_ptr(), nn.data_ptr(),
                              st)
            torch.cuda.synchronize()
            H[a:a + m] = hh[:m].cpu().numpy().view(np.uint64)
            NH[a:a + m] = nn[:m].cpu().numpy().view(np.uint32)
    return H, NH


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=1000)
    ap.add_argument("--genome-bp", type=int, default=5_000_000)
    ap.add_argument("--family-size", type=int, default=100)
    ap.add_argument("--sketch", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0xD2E9)
    ap.add_argument("--method", default="average")
    ap.add_argument("--P-ani", type=float, default=0.9)
    ap.add_argument("--processors", type=int, default=16)
    ap.add_argument("--reference-leg", action="store_true")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from drep_amd import _lib, d_cluster
    from drep_amd.mash_io import MashReference, write_msh
    from drep_amd.store import store_primary_linkage

    N, s = a.genomes, a.sketch
    wd = a.workdir or tempfile.mkdtemp(prefix="dropin_", dir=os.environ.get("TMPDIR", "/tmp"))
    data = os.path.join(wd, "data")
    t = time.perf_counter()
    H, NH = synth_sketches(N, a.genome_bp, a.family_size, s, a.seed)
    synth_s = time.perf_counter() - t
    rng = np.random.default_rng(1)
    names = ["genome_%07d.fna" % i for i in rng.permutation(N)]       # Bdb order != sorted order
    locs = ["/genomes/" + n for n in names]                             # never read: every sketch is cached
    t = time.perf_counter()
    for i, n in enumerate(names):
        d = os.path.join(data, "MASH_files", "sketches", "chunk_%d" % (i // 1000))
        os.makedirs(d, exist_ok=True)
        write_msh(os.path.join(d, n + ".msh"), [MashReference(locs[i], "", a.genome_bp, H[i, :NH[i]])], 21, s, 42)
    cache_write_s = time.perf_counter() - t
    Bdb = pd.DataFrame({"genome": names, "location": locs})
    kwargs = dict(MASH_sketch=str(s), processors=a.processors, groupSize=1000, clusterAlg=a.method, P_ani=a.P_ani)

    # ---- the timed branch (d_cluster.py:170, 177, 185)
    t0 = time.perf_counter()
    Mdb = d_cluster.all_vs_all_MASH(Bdb, data, **kwargs)
    t1 = time.perf_counter()
    stages = dict(d_cluster.STAGE_TIMES)
    Cdb, cluster_ret = d_cluster.cluster_mash_database(Mdb, **kwargs)
    t2 = time.perf_counter()
    store_primary_linkage(data, *cluster_ret)
    t3 = time.perf_counter()
    stages.update({k: v for k, v in d_cluster.STAGE_TIMES.items() if k not in stages})
    if stages.get("sketched_genomes"):
        raise RuntimeError("the timed call re-sketched %d genomes: the cache was not used" % stages["sketched_genomes"])
    out = {
        "what": "Mash branch of cluster_genomes (ref d_cluster.py:168-185) through drep_amd.d_cluster, "
                "sketches cached as .msh (dRep's rerun), CLI kwargs",
        "genomes": N, "genome_bp": a.genome_bp, "family_size": a.family_size, "sketch": s, "method": a.method,
        "P_ani": a.P_ani, "processors": a.processors, "mdb_rows": len(Mdb),
        "branch_s": t3 - t0, "all_vs_all_MASH_s": t1 - t0, "cluster_mash_database_s": t2 - t1,
        "store_primary_linkage_s": t3 - t2, "stages_s": stages,
        "setup": {"synth_and_sketch_s": synth_s, "msh_cache_write_s": cache_write_s},
        "primary_clusters": int(Cdb["primary_cluster"].nunique()),
        "build_id": _lib.build_id(),
    }
    if a.reference_leg:
        import scipy.cluster.hierarchy as sch
        import scipy.spatial.distance as ssd
        Mdb2 = d_cluster.all_vs_all_MASH(Bdb, data, **kwargs)
        r = {}
        t = time.perf_counter()
        Mdb2["dist"] = 1 - Mdb2["similarity"]
        r["dist_update_s"] = time.perf_counter() - t
        t = time.perf_counter()
        lp = Mdb2.pivot(index="genome1", columns="genome2", values="dist")
        r["pandas_pivot_s"] = time.perf_counter() - t
        t = time.perf_counter()
        y = ssd.squareform(np.asarray(lp))
        r["squareform_s"] = time.perf_counter() - t
        t = time.perf_counter()
        Z = sch.linkage(y, method=a.method)
        r["scipy_linkage_s"] = time.perf_counter() - t
        t = time.perf_counter()
        fcl = sch.fcluster(Z, 1 - a.P_ani, criterion="distance")
        Cref = pd.DataFrame({"cluster": fcl, "genome": list(lp.columns)}).rename(columns={"cluster": "primary_cluster"})
        r["fcluster_cdb_s"] = time.perf_counter() - t
        r["total_s"] = sum(r.values())
        ldb = cluster_ret[1]
        pd.testing.assert_frame_equal(ldb, lp, check_exact=True)
        r["linkage_db_identical"] = bool(type(ldb.index) is type(lp.index) and ldb.index.dtype == lp.index.dtype
                                         and np.array_equal(ldb.to_numpy().view(np.uint32), lp.to_numpy().view(np.uint32)))
        r["Z_identical"] = bool(np.array_equal(cluster_ret[0], Z))
        r["Cdb_identical"] = bool(Cdb[["primary_cluster", "genome"]].astype(str).to_dict("list")
                                  == Cref[["primary_cluster", "genome"]].astype(str).to_dict("list"))
        r["mdb_dist_after_identical"] = bool(np.array_equal(Mdb["dist"].to_numpy().view(np.uint32),
                                                            Mdb2["dist"].to_numpy().view(np.uint32)))
        r["speedup_cluster_mash_database"] = r["total_s"] / out["cluster_mash_database_s"]
        out["reference_leg"] = r
        if not (r["linkage_db_identical"] and r["Z_identical"] and r["Cdb_identical"] and r["mdb_dist_after_identical"]):
            print(json.dumps(out), flush=True)
            raise SystemExit("drop-in differs from the reference steps")
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(json.dumps(out, indent=1) + "\n")
    if not a.workdir:
        shutil.rmtree(wd, ignore_errors=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
