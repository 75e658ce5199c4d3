"""Generate the reference-derived golden vectors in tests/golden/ref/.

Run in the build container only (it imports the read-only reference at
/root/reference; the GPU box never has it):

    python3 -B tests/golden/make_golden.py

What it captures, by importing the reference's own Python (Biopython is not
installed, so ``Bio``/``Bio.SeqIO`` are stubbed; nothing on this path uses
them):

* ``all_vs_all_MASH`` (drep/d_cluster.py:481-596) run with ``dry=True`` over
  the reference's fixture ``MASH_table.tsv`` -> the parsed Mdb exactly as the
  reference builds it (dtypes, category order, float32 values, row order).
* ``cluster_mash_database`` (drep/d_cluster.py:598-630) on that Mdb, for the
  CLI default (average) and the function default (single) linkage.  The call at
  d_cluster.py:620 uses positional ``DataFrame.pivot`` arguments, which pandas
  2.x rejects; the script shims ``pivot`` to forward them as keywords (the
  reference's intended semantics), without touching the reference files.

Outputs (small, committed): mdb_parsed.csv, mdb_parsed_dtypes.json,
mdb_after_cluster_<alg>.csv, cdb_<alg>.csv, linkage_<alg>.json.
"""
import json
import os
import shutil
import sys
import tempfile
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ref")


def main():
    sys.path.insert(0, REF)
    bio = types.ModuleType("Bio")
    bio.SeqIO = types.ModuleType("Bio.SeqIO")
    sys.modules["Bio"] = bio
    sys.modules["Bio.SeqIO"] = bio.SeqIO
    import numpy as np
    import pandas as pd

    _pivot = pd.DataFrame.pivot

    def pivot(self, *args, **kw):
        if args:
            kw.update(dict(zip(["index", "columns", "values"], args)))
        return _pivot(self, **kw)

    pd.DataFrame.pivot = pivot
    import drep.d_cluster as dc

    os.makedirs(OUT, exist_ok=True)
    genomes = ["Enterococcus_casseliflavus_EC20.fasta", "Enterococcus_faecalis_T2.fna",
               "Enterococcus_faecalis_TX0104.fa", "Enterococcus_faecalis_YI6-1.fna",
               "Escherichia_coli_Sakai.fna"]
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "MASH_files"))
        shutil.copy(os.path.join(HERE, "MASH_files", "MASH_table.tsv"),
                    os.path.join(tmp, "MASH_files", "MASH_table.tsv"))
        Bdb = pd.DataFrame({"genome": genomes, "location": ["/x/" + g for g in genomes]})
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            Mdb = dc.all_vs_all_MASH(Bdb, tmp, dry=True, exe_loc="mash", processors=1)
    Mdb.to_csv(os.path.join(OUT, "mdb_parsed.csv"), index=False, float_format="%.9g")
    meta = {
        "dtypes": {c: str(t) for c, t in Mdb.dtypes.items()},
        "categories": {g: list(Mdb[g].cat.categories) for g in ("genome1", "genome2")},
        "ordered": {g: bool(Mdb[g].cat.ordered) for g in ("genome1", "genome2")},
        "dist_bits": [int(x) for x in Mdb["dist"].to_numpy().view(np.uint32)],
        "similarity_bits": [int(x) for x in Mdb["similarity"].to_numpy().view(np.uint32)],
    }
    with open(os.path.join(OUT, "mdb_parsed_dtypes.json"), "w") as fh:
        json.dump(meta, fh, indent=1)

    for alg in ("average", "single"):
        db = Mdb.copy()
        Cdb, ret = dc.cluster_mash_database(db, clusterAlg=alg, P_ani=0.9)
        linkage, linkage_db, args = ret
        db.to_csv(os.path.join(OUT, "mdb_after_cluster_%s.csv" % alg), index=False, float_format="%.9g")
        Cdb.to_csv(os.path.join(OUT, "cdb_%s.csv" % alg), index=False)
        with open(os.path.join(OUT, "linkage_%s.json" % alg), "w") as fh:
            json.dump({"linkage": [[float(v).hex() for v in row] for row in linkage],
                       "linkage_repr": [[repr(float(v)) for v in row] for row in linkage],
                       "names": list(linkage_db.columns), "arguments": args,
                       "dist_bits_after": [int(x) for x in db["dist"].to_numpy().view(np.uint32)]},
                      fh, indent=1)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
