"""FASTA ingest + sketch throughput of drephip_sketch_files (host parse/pack
with `threads` threads, H2D, GPU sketch, D2H) on synthetic 5 Mbp genomes
written to a temp dir, plain and gzip.  Not part of the product."""
import gzip, json, os, sys, tempfile, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drep_amd import _lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
L = 5_000_000
threads = int(os.environ.get("INGEST_THREADS", 16))
rng = np.random.default_rng(0)
base = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)]
out = {"genomes": n, "genome_bp": L, "threads": threads}
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    plain, gz = [], []
    for g in range(n):
        seq = base.copy()
        m = rng.random(L) < 0.01
        seq[m] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(m.sum()))]
        lines = b"\n".join(seq[i:i + 80].tobytes() for i in range(0, L, 80))
        txt = b">g%d synthetic\n" % g + lines + b"\n"
        p = os.path.join(td, "g%04d.fna" % g); open(p, "wb").write(txt); plain.append(p)
        if g < n // 4:
            q = p + ".gz"; open(q, "wb").write(gzip.compress(txt, 1)); gz.append(q)
    with _lib.Context(0, 21, 1000, 42) as ctx:
        ctx.sketch_files(plain[:2], threads=threads)                       # warm-up
        for name, files in (("plain", plain), ("gzip", gz)):
            t0 = time.perf_counter()
            h, nh, ln = ctx.sketch_files(files, threads=threads)
            dt = time.perf_counter() - t0
            out[name] = {"files": len(files), "s": dt, "Mbp_per_s": len(files) * L / dt / 1e6,
                         "genomes_per_s": len(files) / dt}
print(json.dumps(out))
