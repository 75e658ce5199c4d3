"""FASTA ingest + sketch of drephip_sketch_files, and the whole drop-in
all_vs_all_MASH, on the reference's test genomes replicated into many files
(plain and gzip).  Reports the host ingest time (read + pack, producer
thread) next to the device time and the wall time of the overlapped pipeline
(the plain set twice: the first call also pins its two batch buffers).
Not part of the product.

usage: python tools/ingest_bench.py [copies_per_genome] > profiles/<round>_ingest.json
"""
import glob
import gzip
import json
import os
import shutil
import sys
import tempfile
import time

import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from drep_amd import _lib, d_cluster  # noqa: E402

copies = int(sys.argv[1]) if len(sys.argv) > 1 else 125
threads = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
src = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "genomes", "*.gz")))
out = {"source": "tests/golden/genomes (4 reference FASTAs) x %d copies each" % copies, "threads": threads}
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    plain, gz = [], []
    for i, f in enumerate(src):
        txt = gzip.open(f).read()
        for c in range(copies):
            p = os.path.join(td, "c%04d_%s" % (c, os.path.basename(f)[:-3]))
            open(p, "wb").write(txt)
            plain.append(p)
        q = os.path.join(td, "z_" + os.path.basename(f))
        shutil.copy(f, q)
        gz.extend([q] * max(1, copies // 4))
    out["files_plain"] = len(plain)
    out["fasta_bytes"] = sum(os.path.getsize(p) for p in plain)
    with _lib.Context(0, 21, 1000, 42) as ctx:
        ctx.sketch_files(plain[:2], threads=threads)                       # warm-up
        for name, files in (("plain_first_call", plain), ("plain", plain), ("gzip", gz)):
            t0 = time.perf_counter()
            h, nh, ln = ctx.sketch_files(files, threads=threads)
            dt = time.perf_counter() - t0
            st = ctx.ingest_stats()
            bases = int(ln.sum())
            out[name] = {"files": len(files), "bases": bases, "wall_s": dt, "Mbp_per_s": bases / dt / 1e6,
                         "library_wall_s": st["wall_s"],
                         "host_read_pack_s": st["produce_s"], "device_s": st["gpu_s"], "batches": st["batches"],
                         "read_parse_thread_s": st["read_thread_s"], "pack_thread_s": st["pack_thread_s"],
                         "overflow_genomes": st["overflow_genomes"],
                         "ingest_only_Mbp_per_s": bases / st["produce_s"] / 1e6,
                         "overlap_note": "wall ~ host read+pack of every batch + the last batch's device work "
                                         "(the other batches' device work runs behind the next batch's ingest)"}
    # the whole drop-in on the plain files: sketch (ingest overlapped) + all-pairs + Mdb
    Bdb = pd.DataFrame({"genome": [os.path.basename(p) for p in plain], "location": plain})
    wd = os.path.join(td, "wd")
    t0 = time.perf_counter()
    Mdb = d_cluster.all_vs_all_MASH(Bdb, wd, processors=threads)
    out["dropin_all_vs_all_MASH"] = {"genomes": len(plain), "wall_s": time.perf_counter() - t0, "mdb_rows": len(Mdb),
                                     "note": "sketch files (+ .msh writing) + HIP all-pairs + float32 Mdb build"}
print(json.dumps(out, indent=1))
