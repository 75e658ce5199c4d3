"""Pin the CPU oracle (oracle/mash_oracle.c) to the reference's own fixtures.

Every golden file here comes from the reference test data
(tests/test_solutions/ecoli_wd/data/MASH_files, tests/genomes) or from
importing the reference Python (tests/golden/make_golden.py).
"""
import glob
import os

import numpy as np
import pytest

import oracle
from drep_amd.mash_io import read_msh

S = 1000


def _fastas(golden):
    return sorted(glob.glob(os.path.join(golden, "genomes", "*.gz")))


def _golden_ref(golden, fasta_gz):
    name = os.path.basename(fasta_gz)[:-3]
    return read_msh(os.path.join(golden, "MASH_files", "sketches", name + ".msh")).references[0]


@pytest.mark.parametrize("idx", range(4))
def test_oracle_sketch_matches_mash_fixture(golden, idx):
    fa = _fastas(golden)[idx]
    ref = _golden_ref(golden, fa)
    h, length = oracle.sketch_fasta(fa, 21, S, 42)
    assert length == ref.length
    assert len(h) == len(ref.hashes) == S
    assert np.array_equal(h, ref.hashes)


def test_oracle_dist_matches_mash_table(golden):
    """25/25 rows of MASH_table.tsv: names, %g dist, %g p-value, c/denom."""
    from scipy.stats import binom
    refs = read_msh(os.path.join(golden, "MASH_files", "ALL.msh")).references
    lines = open(os.path.join(golden, "MASH_files", "MASH_table.tsv")).read().splitlines()
    out = []
    for q in refs:
        for r in refs:
            c, d = oracle.dist_pair(r.hashes, q.hashes, S)
            dist = oracle.mash_distance(c, d)
            ks = 4.0 ** 21
            if c == 0:
                p = 1.0
            else:
                px = 1 / (1 + ks / r.length)
                py = 1 / (1 + ks / q.length)
                rr = px * py / (px + py - px * py)
                M = ks * (px + py) / (1 + rr)
                p = binom.sf(c - 1, int(min(M, S)), rr)
            out.append("%s\t%s\t%s\t%s\t%d/%d" % (r.name, q.name, "%g" % dist, "%g" % p, c, d))
    assert out == lines


def _rand_genome(rng, n_rec, lens, n_frac=0.0, lower_frac=0.0):
    seqs = []
    for L in lens[:n_rec]:
        b = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L)]
        if n_frac:
            m = rng.random(L) < n_frac
            b = b.copy()
            b[m] = ord("N")
        if lower_frac:
            m = rng.random(L) < lower_frac
            b = b.copy()
            b[m] = b[m] + 32
        seqs.append(b.astype(np.uint8))
    return seqs


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_heap_equals_spec(seed):
    """Mash-heap restatement == sort-unique spec, incl. N runs, many records,
    records shorter than k, and repeats."""
    rng = np.random.default_rng(seed)
    lens = [int(x) for x in rng.integers(1, 40000, 12)] + [5, 20, 21, 22]
    seqs = _rand_genome(rng, len(lens), lens, n_frac=0.001)
    seqs.append(np.tile(seqs[0][:500], 30))     # repeats
    seq = np.concatenate(seqs)
    seq = np.where((seq >= 97) & (seq <= 122), seq - 32, seq).astype(np.uint8)
    off = np.concatenate([[0], np.cumsum([len(x) for x in seqs])]).astype(np.uint64)
    for s in (1, 7, 100, 1000, 5000):
        a = oracle.sketch_records(seq, off, 21, s, 42)
        b = oracle.sketch_records(seq, off, 21, s, 42, spec=True)
        assert np.array_equal(a, b), s


def test_oracle_record_boundaries():
    """k-mers never span records: splitting a sequence into two records drops
    exactly the k-mers that crossed the cut."""
    rng = np.random.default_rng(5)
    x = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 3000)].copy()
    whole = oracle.sketch_records(x, np.array([0, 3000], np.uint64), 21, 5000, 42)
    split = oracle.sketch_records(x, np.array([0, 1500, 3000], np.uint64), 21, 5000, 42)
    assert len(whole) == 2980 and len(split) == 2980 - 20


def test_oracle_synthetic_family_distances():
    """The bench's synthetic family gives a spread of shared-hash counts."""
    n, L = 12, 300_000
    h, nh = oracle.sketch_synth(0, n, L, seed=3, family_size=6)
    assert (nh == S).all()
    common, denom = oracle.allpairs(h, nh, S)
    assert (denom == S).all()
    assert common.max() > 100 and common.min() < 20
