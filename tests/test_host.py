"""CPU-only tests: the C ABI library loads and exports every declared symbol,
host-side layout/ingest helpers, .msh I/O, and the Mdb / primary-clustering
host logic against the reference-derived golden vectors (shared-hash counts
from the oracle; no GPU needed)."""
import json
import os
import re

import numpy as np
import pandas as pd
import pytest

import oracle
from drep_amd import _lib
from drep_amd import d_cluster
from drep_amd.mash_io import MashReference, read_msh, write_msh

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S = 1000


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "drephip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = set(re.findall(r"\b(drephip_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    L = _lib.lib()
    for name in declared:
        assert getattr(L, name) is not None
    assert L.drephip_version() >= 100
    # sketch sizes up to 32767 (dRep's -ms/--MASH_sketch is unbounded,
    # drep/argumentParser.py:103; counts and denominators are uint16)
    assert _lib.max_sketch() == 32767


def test_allpairs_kernel_declares_no_static_lds(tmp_path):
    """k_allpairs_q addresses its slot tables at absolute LDS address 0
    (allpairs.hip read_slots, ABS): valid only while the kernel declares no
    static LDS, so its group segment starts with the dynamic region."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "drep_amd", "csrc", "allpairs.hip")
    out = tmp_path / "allpairs.s"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", "-I",
                    os.path.dirname(src), "-o", str(out), src], check=True, capture_output=True, cwd=tmp_path)
    fixed = dict(re.findall(r"\.amdhsa_kernel (\S+)\s.*?\.amdhsa_group_segment_fixed_size (\d+)",
                            out.read_text(), flags=re.S))
    q = {k: int(v) for k, v in fixed.items() if "k_allpairs_q" in k}
    assert q and all(v == 0 for v in q.values()), q


def test_no_cpu_fallback(monkeypatch):
    """The product path fails loudly when the HIP library is missing."""
    import importlib
    monkeypatch.setenv("DREPHIP_LIB", "/nonexistent/libdrephip.so")
    mod = importlib.reload(_lib)
    try:
        with pytest.raises(mod.DrepHipError):
            mod.Context(0, 21, S, 42)
    finally:
        monkeypatch.delenv("DREPHIP_LIB")
        importlib.reload(_lib)


def test_layout_helpers():
    tile = _lib.tile_bases()
    assert tile == 32768
    assert _lib.padded_bases([tile - 1]) == tile
    assert _lib.padded_bases([tile]) == 2 * tile          # >= 1 invalid base after
    assert _lib.padded_bases([10, 20]) == tile
    assert _lib.padded_bases([]) == tile


def test_distance_lut_matches_oracle():
    lut = _lib.distance_lut(S)
    for c in (0, 1, 3, 500, 561, 905, 999, 1000):
        assert lut[c] == oracle.mash_distance(c, S)


def test_fasta_info_matches_oracle_reader(golden):
    import glob
    for fa in sorted(glob.glob(os.path.join(golden, "genomes", "*.gz"))):
        info = _lib.fasta_info(fa)
        seq, off, ln = oracle.read_fasta(fa)
        assert info["length"] == ln
        assert info["n_records"] == len(off) - 1
        reclen = np.diff(off)
        assert info["padded"] == _lib.padded_bases(reclen)


def test_fasta_parser_edge_cases(tmp_path):
    """kseq semantics: text before the first header ignored, CRLF, blank
    lines, lowercase, empty records, gzip."""
    import gzip
    txt = b"junk line\n>r1 desc\r\nACGTac\r\n\r\ngtNN\n>r2\n>r3\nTTTT\n"
    p = tmp_path / "x.fa"
    p.write_bytes(txt)
    pg = tmp_path / "x.fa.gz"
    pg.write_bytes(gzip.compress(txt))
    for path in (p, pg):
        info = _lib.fasta_info(str(path))
        seq, off, ln = oracle.read_fasta(str(path))
        assert bytes(seq) == b"ACGTACGTNNTTTT"
        assert list(off) == [0, 10, 10, 14]
        assert info["length"] == 14 and info["n_records"] == 3


def test_msh_roundtrip_and_fixture(golden, tmp_path):
    m = read_msh(os.path.join(golden, "MASH_files", "ALL.msh"))
    assert (m.kmer, m.sketch_size, m.seed) == (21, S, 42)
    assert len(m.references) == 5
    out = tmp_path / "copy.msh"
    write_msh(str(out), m.references, 21, S, 42)
    m2 = read_msh(str(out))
    assert len(m2.references) == 5
    for a, b in zip(m.references, m2.references):
        assert (a.name, a.comment, a.length) == (b.name, b.comment, b.length)
        assert np.array_equal(a.hashes, b.hashes)
    one = tmp_path / "one.msh"
    write_msh(str(one), [MashReference("x", "", 7, np.array([], np.uint64))], 21, 3, 7)
    r = read_msh(str(one))
    assert (r.kmer, r.sketch_size, r.seed, len(r.references[0].hashes)) == (21, 3, 7, 0)


def _square(vec, N, diag):
    """Symmetric N x N matrix of a condensed vector (scipy order) and a diagonal."""
    M = np.zeros((N, N), dtype=vec.dtype)
    iu = np.triu_indices(N, 1)
    M[iu] = vec
    M = M + M.T
    M[np.arange(N), np.arange(N)] = diag
    return M


def _fixture_condensed(golden):
    refs = read_msh(os.path.join(golden, "MASH_files", "ALL.msh")).references
    H = np.stack([r.hashes for r in refs])
    NH = np.full(len(refs), S, np.uint32)
    c, d = oracle.allpairs(H, NH, S)
    names = [os.path.basename(r.name) for r in refs]
    return d_cluster.CondensedMash(names, [r.name for r in refs], c, d, NH,
                                   np.array([r.length for r in refs], np.uint64), S)


def test_mdb_from_condensed_matches_reference_parse(golden):
    cm = _fixture_condensed(golden)
    Mdb = d_cluster.mdb_from_condensed(cm.names, cm.common, cm.denom, cm.nhash, cm.s)
    meta = json.load(open(os.path.join(golden, "ref", "mdb_parsed_dtypes.json")))
    exp = pd.read_csv(os.path.join(golden, "ref", "mdb_parsed.csv"))
    assert {c: str(t) for c, t in Mdb.dtypes.items()} == meta["dtypes"]
    for g in ("genome1", "genome2"):
        assert list(Mdb[g].cat.categories) == meta["categories"][g]
        assert list(Mdb[g].astype(str)) == list(exp[g])
    assert list(Mdb["dist"].to_numpy().view(np.uint32)) == meta["dist_bits"]
    assert list(Mdb["similarity"].to_numpy().view(np.uint32)) == meta["similarity_bits"]


@pytest.mark.parametrize("alg", ["average", "single"])
def test_cluster_mash_database_matches_reference(golden, alg):
    cm = _fixture_condensed(golden)
    Mdb = d_cluster.mdb_from_condensed(cm.names, cm.common, cm.denom, cm.nhash, cm.s)
    Cdb, ret = d_cluster.cluster_mash_database(Mdb, clusterAlg=alg, P_ani=0.9, gpu=None)
    exp = pd.read_csv(os.path.join(golden, "ref", "cdb_%s.csv" % alg))
    assert Cdb.to_dict("list") == exp.to_dict("list")
    link = json.load(open(os.path.join(golden, "ref", "linkage_%s.json" % alg)))
    assert [[float(v).hex() for v in row] for row in ret[0]] == link["linkage"]
    assert ret[2] == link["arguments"]
    # in-place update of Mdb['dist'] exactly as the reference leaves it
    assert list(Mdb["dist"].to_numpy().view(np.uint32)) == link["dist_bits_after"]
    # the condensed path (no N^2 table) gives the same linkage and clusters
    Cdb2, ret2 = d_cluster.cluster_mash_condensed(cm, clusterAlg=alg, P_ani=0.9, gpu=None)
    assert Cdb2.to_dict("list") == exp.to_dict("list")
    assert np.array_equal(ret2[0], ret[0])


def test_condensed_clustering_equals_pivot_path_unsorted_names():
    """Random synthetic family, names deliberately not in sorted order."""
    n = 30
    h, nh = oracle.sketch_synth(0, n, 150_000, seed=21, family_size=8, threads=4)
    c, d = oracle.allpairs(h, nh, S)
    names = ["g%03d.fa" % ((i * 7) % n) for i in range(n)]
    cm = d_cluster.CondensedMash(names, names, c, d, nh, np.full(n, 150_000, np.uint64), S)
    Mdb = d_cluster.mdb_from_condensed(names, c, d, nh, S)
    for alg in ("average", "single", "complete"):
        Cdb, ret = d_cluster.cluster_mash_database(Mdb.copy(), clusterAlg=alg, P_ani=0.95, gpu=None)
        Cdb2, ret2 = d_cluster.cluster_mash_condensed(cm, clusterAlg=alg, P_ani=0.95, gpu=None)
        assert np.array_equal(ret[0], ret2[0])
        assert Cdb.to_dict("list") == Cdb2.to_dict("list")


def test_write_mash_table_matches_fixture(golden, tmp_path):
    cm = _fixture_condensed(golden)
    out = tmp_path / "MASH_table.tsv"
    d_cluster.write_mash_table(str(out), cm)
    assert out.read_text() == open(os.path.join(golden, "MASH_files", "MASH_table.tsv")).read()


def test_dry_run_parses_existing_table(golden, tmp_path):
    import shutil
    os.makedirs(tmp_path / "MASH_files")
    shutil.copy(os.path.join(golden, "MASH_files", "MASH_table.tsv"), tmp_path / "MASH_files")
    names = sorted(os.path.basename(r.name) for r in
                   read_msh(os.path.join(golden, "MASH_files", "ALL.msh")).references)
    Bdb = pd.DataFrame({"genome": names, "location": ["/x/" + n for n in names]})
    Mdb = d_cluster.all_vs_all_MASH(Bdb, str(tmp_path), dry=True)
    meta = json.load(open(os.path.join(golden, "ref", "mdb_parsed_dtypes.json")))
    assert list(Mdb["dist"].to_numpy().view(np.uint32)) == meta["dist_bits"]


def _np_pack(recs, tile):
    """numpy restatement of the packed layout (include/drephip.h) for one genome."""
    span = sum(len(r) for r in recs) + max(len(recs) - 1, 0)
    P = ((span + 1 + tile - 1) // tile) * tile
    bases = np.full(P, 255, np.uint8)
    pos = 0
    for i, r in enumerate(recs):
        bases[pos:pos + len(r)] = r
        pos += len(r) + 1
    lut = np.full(256, 4, np.uint8)
    for ch, c in zip(b"ACGTacgt", [0, 1, 2, 3, 0, 1, 2, 3]):
        lut[ch] = c
    code = lut[bases]
    ok = code < 4
    c2 = np.where(ok, code, 0).astype(np.uint32).reshape(-1, 16)
    codes = (c2 << (2 * np.arange(16, dtype=np.uint32))).sum(axis=1, dtype=np.uint64).astype(np.uint32)
    v = ok.astype(np.uint32).reshape(-1, 32)
    valid = (v << np.arange(32, dtype=np.uint32)).sum(axis=1, dtype=np.uint64).astype(np.uint32)
    return P, codes, valid


def test_fasta_pack_matches_numpy_layout(tmp_path, golden):
    """Host packer (drephip_fasta_pack) == numpy restatement of the layout, on
    a real multi-record genome with N runs and on a synthetic edge case file."""
    import ctypes as C
    import glob
    rng = np.random.default_rng(2)
    A = np.frombuffer(b"ACGTacgtNRY", dtype=np.uint8)
    recs = [A[rng.integers(0, len(A), n)] for n in (1, 31, 32, 33, 5000, 0, 70000)]
    txt = b"".join(b">r%d\n" % i + b"\n".join(bytes(r[j:j + 61]) for j in range(0, len(r), 61)) + b"\n"
                   for i, r in enumerate(recs))
    p = tmp_path / "e.fa"
    p.write_bytes(txt)
    fas = [str(p)] + sorted(glob.glob(os.path.join(golden, "genomes", "*.gz")))[1:2]
    tile = _lib.tile_bases()
    L = _lib.lib()
    for fa in fas:
        seq, off, ln = oracle.read_fasta(fa)
        recs_o = [seq[off[i]:off[i + 1]] for i in range(len(off) - 1)]
        if fa == str(p):   # oracle upper-cases; the packer accepts either case
            recs_o = [np.array(r) for r in recs]
        P, want_c, want_v = _np_pack(recs_o, tile)
        codes = np.zeros((tile + P) // 16, np.uint32)
        valid = np.zeros((tile + P) // 32, np.uint32)
        length = C.c_uint64(0)
        nk = C.c_uint64(0)
        rc = L.drephip_fasta_pack(fa.encode(), 21, codes, valid, tile, tile + P, C.byref(length), C.byref(nk))
        assert rc == 0
        assert np.array_equal(codes[tile // 16:], want_c)
        assert np.array_equal(valid[tile // 32:], want_v)
        assert not codes[:tile // 16].any() and not valid[:tile // 32].any()
        assert length.value == sum(len(r) for r in recs_o)


def _messy_fasta(rng, n_rec, big):
    """FASTA bytes with kseq corner cases, and the records kseq reads from it:
    random line lengths (1-300, so sequence lines straddle the reader's
    64-byte chunks and 4 MiB blocks), CRLF on some lines, blank lines,
    lowercase, N/IUPAC bytes, '\r' inside lines, long headers, text before the
    first header, FASTQ records whose '+' line ends the sequence."""
    A = np.frombuffer(b"ACGTacgtNRYKM", dtype=np.uint8)
    out, recs = [b"preamble text\n\n"], []
    for r in range(n_rec):
        L = int(rng.integers(0, 3_000_000 if big else 20_000))
        seq = A[rng.integers(0, len(A), L)].copy()
        seq[rng.random(L) < 1e-4] = ord("\r")                  # '\r' inside a line is a (bad) base
        fastq = r % 5 == 4
        out.append((b"@" if fastq else b">") + b"rec%d " % r + b"x" * int(rng.integers(0, 500)) + b"\n")
        kept, i = [], 0
        while i < L:
            w = int(rng.integers(1, 301))
            line = seq[i:i + w].tobytes()
            i += w
            if line.endswith(b"\r"):                              # would be eaten as CRLF
                line = line[:-1] + b"A"
            kept.append(line)
            out.append(line + (b"\r\n" if rng.random() < 0.2 else b"\n"))
            if rng.random() < 0.02:
                out.append(b"\n")
        if fastq:                     # quality lines may start with '@', '>' or '+' (kseq counts them)
            Q = np.frombuffer(b"@>+!#I5?", dtype=np.uint8)
            q = Q[rng.integers(0, len(Q), len(b"".join(kept)))].tobytes()
            out.append(b"+rec%d\n" % r)
            i = 0
            while True:
                w = int(rng.integers(1, 120))
                out.append(q[i:i + w] + b"\n")
                i += w
                if i >= len(q):
                    break
        recs.append(np.frombuffer(b"".join(kept), dtype=np.uint8))
    return b"".join(out), recs


@pytest.mark.parametrize("seed,n_rec,big", [(1, 12, False), (2, 40, False), (3, 4, True)])
def test_fasta_reader_and_packer_on_messy_files(tmp_path, seed, n_rec, big):
    """The SIMD FASTA reader + packer (drephip_fasta_pack) against a direct
    restatement of kseq's rules and the numpy layout, plain and gzip."""
    import ctypes as C
    import gzip
    rng = np.random.default_rng(seed)
    txt, recs = _messy_fasta(rng, n_rec, big)
    tile = _lib.tile_bases()
    P, want_c, want_v = _np_pack(recs, tile)
    L = _lib.lib()
    for name, data in (("m.fa", txt), ("m.fa.gz", gzip.compress(txt, 1))):
        path = tmp_path / name
        path.write_bytes(data)
        codes = np.zeros((tile + P) // 16, np.uint32)
        valid = np.zeros((tile + P) // 32, np.uint32)
        length = C.c_uint64(0)
        nk = C.c_uint64(0)
        rc = L.drephip_fasta_pack(str(path).encode(), 21, codes, valid, tile, tile + P, C.byref(length), C.byref(nk))
        assert rc == 0, name
        assert length.value == sum(len(r) for r in recs), name
        assert np.array_equal(codes[tile // 16:], want_c), name
        assert np.array_equal(valid[tile // 32:], want_v), name


def test_device_list_and_balanced_shards(monkeypatch):
    """Multi-device drop-in plumbing (no GPU): the `gpus` kwarg forms and the
    byte-balanced contiguous genome shards."""
    from drep_amd.d_cluster import _balanced_shards, _devices
    monkeypatch.delenv("DREPHIP_DEVICES", raising=False)
    monkeypatch.delenv("DREPHIP_DEVICE", raising=False)
    assert _devices({}) == [0]
    assert _devices({"gpu": 3}) == [3]
    assert _devices({"gpus": 4}) == [0, 1, 2, 3]
    assert _devices({"gpus": "0,2,5"}) == [0, 2, 5]
    assert _devices({"gpus": [1, 1]}) == [1, 1]
    monkeypatch.setenv("DREPHIP_DEVICES", "6,7")
    assert _devices({"gpu": 0}) == [6, 7]
    rng = np.random.default_rng(0)
    for n_items, n_dev in [(0, 3), (1, 4), (5, 5), (100, 8), (1000, 3)]:
        w = rng.integers(1, 1000, n_items)
        sh = _balanced_shards(w, n_dev)
        assert len(sh) == n_dev
        assert sum(sh, []) == list(range(n_items))           # contiguous cover, in order
        if n_items >= 100:
            tot = [w[s].sum() for s in sh]
            assert max(tot) - min(tot) <= 2 * w.max()


@pytest.mark.parametrize("partial", [False, True])
def test_condensed_store_roundtrip(tmp_path, partial):
    """drep_amd.store: the condensed Mash result and the reference-format
    primary_linkage pickle round-trip, and the long-form Mdb rebuilt from the
    stored counts equals the one built before storing."""
    from drep_amd.d_cluster import CondensedMash, cluster_mash_condensed, mdb_from_condensed
    from drep_amd.store import load_condensed, load_primary_linkage, store_condensed, store_primary_linkage
    rng = np.random.default_rng(1)
    N, s = 12, 1000
    c = rng.integers(0, s + 1, N * (N - 1) // 2).astype(np.uint16)
    d = np.full(len(c), s, np.uint16)
    nh = np.full(N, s, np.uint32)
    if partial:
        d[::3] = 700
        c = np.minimum(c, d)
        nh[2] = 650
    names = ["g%02d.fa" % i for i in rng.permutation(N)]
    cm = CondensedMash(names, ["/x/" + n for n in names], c, d, nh, np.arange(N, dtype=np.uint64) * 1000, s)
    store_condensed(str(tmp_path), cm)
    assert os.path.exists(tmp_path / "MASH_files" / "condensed" / "denom.npy") == partial
    back = load_condensed(str(tmp_path))
    assert back.names == cm.names and back.locations == cm.locations and back.s == s
    for a in ("common", "denom", "nhash", "length"):
        assert np.array_equal(np.asarray(getattr(back, a)), getattr(cm, a)), a
    m0 = mdb_from_condensed(cm.names, cm.common, cm.denom, cm.nhash, s)
    m1 = mdb_from_condensed(back.names, back.common, back.denom, back.nhash, s)
    assert m0.equals(m1)
    cdb, (Z, db, args) = cluster_mash_condensed(back, clusterAlg="average", P_ani=0.9, gpu=None)
    store_primary_linkage(str(tmp_path), Z, db, args)
    pl = load_primary_linkage(str(tmp_path))
    assert np.array_equal(pl["linkage"], Z) and pl["db"] is None and pl["arguments"] == args
    assert set(pl) == {"linkage", "db", "arguments"}          # WorkDirectory.import_clusters keys


KSEQ_CASES = {
    # text before the first header, a '>' in the middle of it starts a record
    "hunt_midline": b"junk >hdr one\nACGT\nacgtN\n>two\nGGGG\n",
    # FASTQ quality lines starting with '@', '>' and '+' are quality, not headers
    "fastq_quality_lookalikes": b"@r1\nACGTACGT\n+\n@>+!\n@@II\n@r2 x\nTTTT\n+r2\n>>>>\n",
    # quality longer than the sequence: kseq_read returns -2, the record and the rest are dropped
    "fastq_long_quality": b"@a\nACGT\n+\nIIII\n@b\nCCCC\n+\nIIIIII\n@c\nGGGG\n+\nIIII\n",
    # quality cut short by EOF: that record is dropped
    "fastq_short_quality": b">f\nAAAACCCC\n@q\nACGTACGT\n+\nIII\n",
    # '+' line and then EOF: no quality, dropped
    "fastq_plus_eof": b">f\nAAAA\n@q\nACGT\n+",
    # '>' as the very last byte: no record
    "gt_last_byte": b">f\nACGT\n>",
    # header without newline at EOF: an empty record
    "header_eof": b">f\nACGT\n>g",
    # empty FASTQ record, nothing after its '+' line
    "fastq_empty_record": b">f\nACGT\n@e\n+\n",
    # after a FASTQ record anything up to the next '>'/'@' is skipped, mid-line too
    "after_fastq_hunt": b"@a\nAC\n+\nII\nnoise x@b\nGGTT\n",
    # CRLF everywhere, blank lines, a line of only '\r'
    "crlf": b">a\r\nACG\r\n\r\nTTA\r\n\n@b\r\nAC\r\n+\r\nII\r\n",
}


@pytest.mark.parametrize("case", sorted(KSEQ_CASES))
def test_fasta_reader_kseq_corner_cases_vs_oracle(tmp_path, case):
    """The SIMD reader (drephip_fasta_info / _pack) and the oracle's byte-level
    restatement of kseq_read agree on kseq's corner cases: header hunting
    anywhere, FASTQ quality lines that look like headers, quality-length
    errors that end the file, EOF inside headers and quality."""
    import ctypes as C
    import gzip
    tile = _lib.tile_bases()
    L = _lib.lib()
    for name, data in (("k.fq", KSEQ_CASES[case]), ("k.fq.gz", gzip.compress(KSEQ_CASES[case]))):
        path = tmp_path / name
        path.write_bytes(data)
        seq, off, ln = oracle.read_fasta(str(path))
        recs = [seq[off[i]:off[i + 1]] for i in range(len(off) - 1)]
        info = _lib.fasta_info(str(path))
        assert info["n_records"] == len(recs), (case, name, info, [bytes(r) for r in recs])
        assert info["length"] == ln
        P, want_c, want_v = _np_pack(recs, tile)
        codes = np.zeros((tile + P) // 16, np.uint32)
        valid = np.zeros((tile + P) // 32, np.uint32)
        length = C.c_uint64(0)
        nk = C.c_uint64(0)
        assert L.drephip_fasta_pack(str(path).encode(), 21, codes, valid, tile, tile + P, C.byref(length),
                                    C.byref(nk)) == 0
        assert np.array_equal(codes[tile // 16:], want_c) and np.array_equal(valid[tile // 32:], want_v), case
    expect = {"hunt_midline": [b"ACGTACGTN", b"GGGG"], "fastq_quality_lookalikes": [b"ACGTACGT", b"TTTT"],
              "fastq_long_quality": [b"ACGT"], "fastq_short_quality": [b"AAAACCCC"],
              "fastq_plus_eof": [b"AAAA"], "gt_last_byte": [b"ACGT"], "header_eof": [b"ACGT", b""],
              "fastq_empty_record": [b"ACGT", b""], "after_fastq_hunt": [b"AC", b"GGTT"],
              "crlf": [b"ACGTTA", b"AC"]}[case]
    assert [bytes(r) for r in recs] == expect


def test_sharded_job_genome_list_and_cache(tmp_path):
    """drep_amd.distributed's file inputs: a FASTA path list or a dRep Bdb
    table give (names, locations) in Bdb order with basename names
    (d_cluster.py:527, 632); the work directory's cached sketches are found in
    the chunk folders of the drop-in's layout (d_cluster.py:531-542)."""
    import shutil
    import pandas as pd
    from drep_amd.distributed import cached_sketches, read_genome_list
    locs = ["/x/a.fna", "/y/b.fasta", "/x/a.fna", "/z/Escherichia_coli_Sakai.fna"]
    lst = tmp_path / "l.txt"
    lst.write_text("\n".join(locs) + "\n\n")
    names, got = read_genome_list(files=str(lst))
    assert got == ["/x/a.fna", "/y/b.fasta", "/z/Escherichia_coli_Sakai.fna"]
    assert names == ["a.fna", "b.fasta", "Escherichia_coli_Sakai.fna"]
    pd.DataFrame({"genome": ["A", "B", "A", "S"], "location": locs}).to_csv(tmp_path / "Bdb.csv", index=False)
    n2, l2 = read_genome_list(bdb=str(tmp_path / "Bdb.csv"))
    assert n2 == ["A", "B", "S"] and l2 == got
    chunk = tmp_path / "wd" / "MASH_files" / "sketches" / "chunk_1"
    chunk.mkdir(parents=True)
    golden = os.path.join(os.path.dirname(__file__), "golden", "MASH_files", "sketches")
    shutil.copy(os.path.join(golden, "Escherichia_coli_Sakai.fna.msh"), chunk / "Escherichia_coli_Sakai.fna.msh")
    c = cached_sketches(str(tmp_path / "wd"), names, 1000, group_size=2)
    assert list(c) == [2] and len(c[2].hashes) == 1000
    assert cached_sketches(str(tmp_path / "wd"), names, 1000, group_size=1000) == {}
    assert cached_sketches(str(tmp_path / "wd"), names, 500, group_size=2) == {}     # other s: not reused


def test_write_mash_table_vs_line_by_line(tmp_path):
    """The threaded C writer against a line-by-line restatement of `mash dist`'s
    output (query outer, reference inner, %g, common/denom) on a family set
    with partial sketches (denominators < s) and distinct genome lengths."""
    n = 37
    h, nh = oracle.sketch_synth(0, n, 60_000, seed=5, family_size=6, threads=4)
    for g in (3, 17):                                    # partial sketches
        h[g, 400:] = np.iinfo(np.uint64).max
        nh[g] = 400
    c, d = oracle.allpairs(h, nh, S)
    names = ["/data/g%02d.fa" % i for i in range(n)]
    length = np.arange(n, dtype=np.uint64) * 1000 + 60_000
    cm = d_cluster.CondensedMash(names, names, c, d, nh, length, S)
    out = tmp_path / "t.tsv"
    d_cluster.write_mash_table(str(out), cm, threads=3)
    Cm = _square(c, n, np.minimum(nh, S).astype(np.uint16)).astype(np.int64)
    Dm = _square(d, n, np.minimum(nh, S).astype(np.uint16)).astype(np.int64)
    lines = []
    for q in range(n):
        for r in range(n):
            lut = _lib.distance_lut(int(Dm[q, r])) if Dm[q, r] else np.zeros(1)
            p = d_cluster.mash_pvalue(np.array([Cm[q, r]]), np.array([float(length[r])]),
                                      np.array([float(length[q])]), S)[0]
            lines.append("%s\t%s\t%g\t%g\t%d/%d\n" % (names[r], names[q], lut[Cm[q, r]], p, Cm[q, r], Dm[q, r]))
    assert out.read_text() == "".join(lines)


# ------------------------------------------------- sparse linkage (host only)
def _sparse_instance(rng, n, kind):
    """n x n distances in [0, 1] with 1.0 between 'families' (Mash's distance of
    genomes with no shared hash): few distinct values (ties), continuous
    values, values a hair below 1.0 (weighted averages round to 1.0), or no
    pair at 1.0 at all (one component)."""
    fam = rng.integers(0, max(1, n // int(rng.integers(2, 12))), n)
    iu = np.triu_indices(n, 1)
    m = len(iu[0])
    if kind == "ties":
        v = rng.integers(1, 5, m) / 8.0
    elif kind == "cont":
        v = rng.random(m) * 0.9
    elif kind == "near1":
        v = 1.0 - rng.integers(1, 4, m) * 2.0 ** -52
    else:                                   # "dense": every pair below 1.0
        v = rng.integers(1, 50, m) / 64.0
    keep = (fam[iu[0]] == fam[iu[1]]) & (rng.random(m) < rng.random()) if kind != "dense" else np.ones(m, bool)
    if kind == "chance":
        # Mash at scale: families at continuous distances plus a few chance
        # links between unrelated genomes at two distances (one or two shared
        # hashes) -- one component, many ties at the chance level
        v = np.where(fam[iu[0]] == fam[iu[1]], rng.random(m) * 0.2, rng.choice([0.33, 0.30], m))
        keep = (fam[iu[0]] == fam[iu[1]]) | (rng.random(m) < 0.03)
    y = np.ones(m)
    y[keep] = v[keep]
    return y, iu


@pytest.mark.parametrize("rows", ["0", "2"])
@pytest.mark.parametrize("kind", ["ties", "cont", "near1", "dense", "chance"])
def test_linkage_sparse_matches_scipy(kind, rows, monkeypatch):
    """drephip_linkage_sparse (scipy's nn_chain / Prim replayed on the pairs
    below 1.0, every other pair at 1.0) == scipy.cluster.hierarchy.linkage of
    the dense matrix, bit for bit, for every method it serves -- including
    ties, clusters that lose every edge below 1.0 (complete linkage; weighted
    averages rounding up to 1.0) and a set with no pair at 1.0.  Both forms:
    per-component matrices (rows 0) and the sparse-row chain / heap Prim
    (rows 2, the form of one large component)."""
    import scipy.cluster.hierarchy as sch
    monkeypatch.setenv("DREPHIP_LINK_ROWS", rows)
    rng = np.random.default_rng(len(kind))
    for trial in range(60):
        n = int(rng.integers(2, 120))
        y, iu = _sparse_instance(rng, n, kind)
        sel = y < 1.0
        perm = rng.permutation(int(sel.sum()))           # the list order does not matter
        pi, pj, pv = iu[0][sel][perm], iu[1][sel][perm], y[sel][perm]
        if trial % 2:
            pi, pj = pj, pi                               # nor which end comes first
        for method in ("single", "complete", "average", "weighted"):
            Zs = sch.linkage(y, method=method)
            Z = _lib.linkage_sparse(n, pi, pj, pv, method)
            assert np.array_equal(Z, Zs), (kind, trial, n, method, np.argwhere(Z != Zs)[:4])


@pytest.mark.parametrize("rows", ["0", "2"])
def test_linkage_sparse_rejects_bad_lists(rows, monkeypatch):
    """A pair listed twice, a value at or above 1.0 (not a sparse entry), an
    index out of range or i == j is refused, not silently clustered (both
    forms)."""
    monkeypatch.setenv("DREPHIP_LINK_ROWS", rows)
    with pytest.raises(_lib.DrepHipError, match="twice"):
        _lib.linkage_sparse(4, [0, 1], [1, 0], [0.5, 0.5], "average")
    with pytest.raises(_lib.DrepHipError, match="twice"):
        _lib.linkage_sparse(4, [0, 0], [1, 1], [0.5, 0.25], "single")
    with pytest.raises(_lib.DrepHipError, match=r"\[0, 1\)"):
        _lib.linkage_sparse(4, [0], [1], [1.0], "average")
    with pytest.raises(_lib.DrepHipError, match=r"\[0, 1\)"):
        _lib.linkage_sparse(4, [0], [1], [np.nan], "complete")
    with pytest.raises(_lib.DrepHipError, match="range"):
        _lib.linkage_sparse(4, [0], [4], [0.5], "average")
    with pytest.raises(_lib.DrepHipError, match="range"):
        _lib.linkage_sparse(4, [2], [2], [0.5], "average")
    with pytest.raises(KeyError):
        _lib.linkage_sparse(4, [0], [1], [0.5], "ward")
    assert _lib.linkage_sparse(1, [], [], [], "average").shape == (0, 4)
    Z = _lib.linkage_sparse(3, [], [], [], "average")          # no pair below 1.0
    assert Z.tolist() == [[0, 1, 1.0, 2], [2, 3, 1.0, 3]]


def test_gzip_reader_libdeflate_equals_zlib(golden, tmp_path):
    """The whole-file libdeflate inflate and zlib's streaming gzread give the
    same packed genome (and the same errors) on: the reference's gzipped
    genomes, a file of several gzip members with trailing junk (zlib's
    gzread semantics), a gzipped FASTQ and a truncated member."""
    import glob
    import gzip
    import subprocess
    import sys
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fas = sorted(glob.glob(os.path.join(golden, "genomes", "*.gz")))
    raw = gzip.decompress(open(fas[1], "rb").read())
    third = len(raw) // 3
    mm = tmp_path / "multi.fa.gz"
    mm.write_bytes(gzip.compress(raw[:third]) + gzip.compress(raw[third:2 * third]) +
                   gzip.compress(raw[2 * third:]) + b"trailing junk")
    fq = tmp_path / "reads.fq.gz"
    fq.write_bytes(gzip.compress(b"@r1\nACGTACGTACGTACGTACGTACGTAC\n+\nIIIIIIIIIIIIIIIIIIIIIIIIII\n"
                                 b"@r2\nTTTTGGGGCCCCAAAATTTTGGGGCCCC\n+\nIIIIIIIIIIIIIIIIIIIIIIIIIIII\n"))
    tr = tmp_path / "truncated.fa.gz"
    full = gzip.compress(raw)
    tr.write_bytes(full[:len(full) // 2])
    files = fas + [str(mm), str(fq), str(tr)]
    code = r"""
import ctypes as C, hashlib, json, sys
import numpy as np
sys.path.insert(0, %r)
from drep_amd import _lib
L = _lib.lib(); tile = _lib.tile_bases(); out = []
for fa in %r:
    try:
        info = _lib.fasta_info(fa)
    except _lib.DrepHipError as e:
        out.append("error"); continue
    P = info["padded"]
    codes = np.zeros((tile + P) // 16, np.uint32); valid = np.zeros((tile + P) // 32, np.uint32)
    ln, nk = C.c_uint64(0), C.c_uint64(0)
    rc = L.drephip_fasta_pack(fa.encode(), 21, codes, valid, tile, tile + P, C.byref(ln), C.byref(nk))
    out.append([rc, ln.value, nk.value, hashlib.sha1(codes.tobytes() + valid.tobytes()).hexdigest()])
print(json.dumps(out))
""" % (ROOT, files)
    res = []
    for no_ld in (False, True):
        env = dict(os.environ)
        env.pop("DREPHIP_NO_LIBDEFLATE", None)
        if no_ld:
            env["DREPHIP_NO_LIBDEFLATE"] = "1"
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
        res.append(json.loads(r.stdout))
    assert res[0] == res[1]
    assert res[0][len(fas)] == res[0][1]            # the members concatenated: the original file
    assert res[0][-1] == "error" or res[0][-1][0] != 0 or res[0][-1][1] < len(raw)


# ------------------------------------------ Mdb table and pivot (host, native)
def _mdb_numpy(names, common, denom, s):
    """The Mdb as the earlier pure-numpy restatement built it: squareform of the
    float32 distances, tile/repeat of the category codes."""
    import scipy.spatial.distance as ssd
    N = len(names)
    dist = ssd.squareform(d_cluster.mash_distance_float32(common, denom), checks=False).reshape(-1)
    cats = sorted(set(names))
    codes = np.array([cats.index(n) for n in names])
    g1 = pd.Categorical.from_codes(np.tile(codes, N), categories=cats, ordered=True)
    g2 = pd.Categorical.from_codes(np.repeat(codes, N), categories=cats, ordered=True)
    Mdb = pd.DataFrame({"genome1": g1, "genome2": g2, "dist": dist})
    Mdb["similarity"] = 1 - Mdb["dist"]
    return Mdb


@pytest.mark.parametrize("n,partial", [(2, False), (37, True), (130, False), (300, True)])
def test_mdb_from_condensed_native_equals_numpy(n, partial):
    """drephip_mdb_square against the numpy restatement: every cell's float32
    bits, the category codes and dtypes (int8 codes below 127 names, int16
    above), partial sketches (one table per denominator), unsorted names."""
    rng = np.random.default_rng(n)
    npairs = n * (n - 1) // 2
    denom = np.full(npairs, S, np.uint16)
    if partial:
        denom[rng.random(npairs) < 0.2] = rng.integers(0, 700, 1)[0]
        denom[rng.random(npairs) < 0.05] = 0
    common = np.minimum(rng.integers(0, S + 1, npairs), denom).astype(np.uint16)
    names = ["g%04d.fa" % i for i in rng.permutation(n)]
    got = d_cluster.mdb_from_condensed(names, common, denom, None, S, threads=3)
    want = _mdb_numpy(names, common, denom, S)
    pd.testing.assert_frame_equal(got, want, check_exact=True)
    for c in ("dist", "similarity"):
        assert np.array_equal(got[c].to_numpy().view(np.uint32), want[c].to_numpy().view(np.uint32))
    assert got["genome1"].cat.codes.dtype == (np.int8 if n < 127 else np.int16)
    bad = common.copy()
    bad[0] = S + 1 if not partial else denom[0] + 1
    with pytest.raises(_lib.DrepHipError, match="exceeds"):
        d_cluster.mdb_from_condensed(names, bad, denom, None, S)


def _pivot_ref(db):
    return db.pivot(index="genome1", columns="genome2", values="dist")


def _assert_pivot_equal(got, want):
    pd.testing.assert_frame_equal(got, want, check_exact=True)
    for a, b in ((got.index, want.index), (got.columns, want.columns)):
        assert type(a) is type(b) and a.name == b.name and a.dtype == b.dtype
    assert np.array_equal(got.to_numpy().view(np.uint32), want.to_numpy().view(np.uint32))


def test_pivot_native_equals_pandas():
    """_pivot_dist (drephip_pivot_scan/fill) against pandas' own pivot on the
    layouts a Mdb can have: all_vs_all_MASH's (blocked transpose), rows
    shuffled (scatter), rows missing (NaN cells), unused categories, genome
    names with 1-byte and 2-byte codes; duplicates raise pandas' error; tables
    outside the fast path (unsorted categories, float64 dist, object columns)
    go through pandas and still match."""
    rng = np.random.default_rng(3)
    for n in (1, 2, 5, 140):
        npairs = n * (n - 1) // 2
        common = rng.integers(0, 40, npairs).astype(np.uint16)
        names = ["g%03d.fa" % i for i in rng.permutation(n)]
        Mdb = d_cluster.mdb_from_condensed(names, common, np.full(npairs, S, np.uint16), None, S)
        Mdb["dist"] = 1 - Mdb["similarity"]
        _assert_pivot_equal(d_cluster._pivot_dist(Mdb), _pivot_ref(Mdb))
        if n < 5:
            continue
        sh = Mdb.sample(frac=1.0, random_state=1).reset_index(drop=True)        # any row order
        _assert_pivot_equal(d_cluster._pivot_dist(sh), _pivot_ref(sh))
        miss = sh.iloc[3:].reset_index(drop=True)                               # missing cells -> NaN
        _assert_pivot_equal(d_cluster._pivot_dist(miss), _pivot_ref(miss))
        part = Mdb[Mdb["genome1"] != names[0]].reset_index(drop=True)          # a name only in genome2
        _assert_pivot_equal(d_cluster._pivot_dist(part), _pivot_ref(part))
        extra = Mdb.copy()                                                      # an unused category
        for g in ("genome1", "genome2"):
            extra[g] = extra[g].cat.add_categories(["zzz_unused.fa"])
        _assert_pivot_equal(d_cluster._pivot_dist(extra), _pivot_ref(extra))
        dup = pd.concat([Mdb, Mdb.iloc[[7]]], ignore_index=True)
        with pytest.raises(ValueError, match="duplicate entries"):
            _pivot_ref(dup)
        with pytest.raises(ValueError, match="duplicate entries"):
            d_cluster._pivot_dist(dup)
        for other in (Mdb.astype({"dist": np.float64}),
                      Mdb.assign(genome1=Mdb["genome1"].astype(str), genome2=Mdb["genome2"].astype(str)),
                      Mdb.assign(genome1=Mdb["genome1"].cat.reorder_categories(sorted(names, reverse=True)),
                                 genome2=Mdb["genome2"].cat.reorder_categories(sorted(names, reverse=True)))):
            _assert_pivot_equal(d_cluster._pivot_dist(other), _pivot_ref(other))


def test_cluster_mash_database_host_path_equals_reference_steps():
    """cluster_mash_database(gpu=None) -- the native pivot, then scipy -- equals
    the reference's steps literally (d_cluster.py:619-623, 445-459) on a
    shuffled family set: linkage_db, Z, Cdb and the in-place dist bits; an
    asymmetric table logs and raises squareform's error."""
    import scipy.cluster.hierarchy as sch
    import scipy.spatial.distance as ssd
    n = 60
    h, nh = oracle.sketch_synth(0, n, 120_000, seed=9, family_size=6, threads=4)
    c, d = oracle.allpairs(h, nh, S)
    names = ["g%03d.fa" % i for i in np.random.default_rng(2).permutation(n)]
    Mdb = d_cluster.mdb_from_condensed(names, c, d, nh, S)
    ref = Mdb.copy()
    ref["dist"] = 1 - ref["similarity"]
    lp = ref.pivot(index="genome1", columns="genome2", values="dist")
    Z = sch.linkage(ssd.squareform(np.asarray(lp)), method="average")
    fcl = sch.fcluster(Z, 1 - 0.95, criterion="distance")
    Cdb, (Zg, ldb, args) = d_cluster.cluster_mash_database(Mdb, clusterAlg="average", P_ani=0.95, gpu=None)
    _assert_pivot_equal(ldb, lp)
    assert np.array_equal(Zg, Z)
    assert list(Cdb["primary_cluster"]) == list(fcl) and list(Cdb["genome"]) == list(lp.columns)
    assert np.array_equal(Mdb["dist"].to_numpy().view(np.uint32), ref["dist"].to_numpy().view(np.uint32))
    asym = Mdb.copy()
    asym.loc[5, "similarity"] = np.float32(0.5)
    with pytest.raises(ValueError, match="symmetric"):
        d_cluster.cluster_mash_database(asym, clusterAlg="average", gpu=None)
