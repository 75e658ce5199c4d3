"""Drop-in for the Mash half of dRep's primary clustering, on MI355X.

Mirrors the reference functions of ``drep/d_cluster.py`` that sit on the hot
path -- same names, arguments, return values and side effects on the work
directory -- with the external ``mash sketch`` / ``mash paste`` /
``mash dist`` processes replaced by libdrephip.so (HIP kernels, gfx950):

===============================  ==========================================
reference (drep/d_cluster.py)    here
===============================  ==========================================
all_vs_all_MASH       481-596    :func:`all_vs_all_MASH`
cluster_mash_database 598-630    :func:`cluster_mash_database` (its
  cluster_hierarchical 429-461 /  linkage + fcluster + Cdb steps inline)
  _gen_cdb_from_fclust 463-479
_get_genome_name_from_fasta 632  :func:`_get_genome_name_from_fasta`
===============================  ==========================================

dRep's own ``load_genomes`` (1483-1518) builds the Bdb these functions take;
it is not on the hot path and stays dRep's.

Beyond the reference (needed at 10^4-10^5 genomes, where an N^2-row Mdb does
not fit): :func:`all_vs_all_MASH_condensed` returns the condensed
``common``/``denom`` vectors and :func:`mdb_from_condensed` /
:func:`cluster_mash_condensed` build the Mdb / primary clusters from them with
the same float32 arithmetic the reference applies; with ``gpu=`` the linkage
itself (scipy's algorithm, bit-identical Z) runs on the GPU.
"""
from __future__ import annotations

import io
import logging
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import pandas as pd
import scipy.cluster.hierarchy
import scipy.spatial.distance as ssd

from . import _lib
from .mash_io import MashReference, read_msh, write_msh
from .parallel import cond_start, row_partition, segment_size

MASH_K = 21          # Mash default, never overridden by dRep (d_cluster.py:543)
MASH_SEED = 42       # Mash default hash seed

# host wall-clock seconds of the stages of the last all_vs_all_MASH /
# cluster_mash_database call in this process (tools/dropin_bench.py reports
# them; nothing reads them on the product path)
STAGE_TIMES: Dict[str, float] = {}


class _Stage:
    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        import time
        self.t0 = time.perf_counter()

    def __exit__(self, *a):
        import time
        STAGE_TIMES[self.name] = time.perf_counter() - self.t0


# --------------------------------------------------------------- genomes
def _get_genome_name_from_fasta(fasta):
    """os.path.basename (reference drep/d_cluster.py:632-642)."""
    return str(os.path.basename(fasta))


# ----------------------------------------------------------- distances
def mash_distance_float32(common: np.ndarray, denom: np.ndarray, k: int = MASH_K) -> np.ndarray:
    """float32 "dist" values exactly as the reference obtains them.

    The reference parses Mash's text output: ``mash dist`` prints the double
    distance with C++ ostream defaults (= ``%g``, 6 significant digits) and
    ``pd.read_csv(..., dtype={'dist': np.float32})`` parses it
    (d_cluster.py:570-581).  Distance is a pure function of (common, denom), so
    the at most (s+1) x (#denominators) distinct values are formatted and
    pushed through the same ``read_csv`` call, then gathered.
    """
    common = np.asarray(common)
    denom = np.asarray(denom)
    out = np.empty(common.shape, dtype=np.float32)
    if common.size == 0:
        return out
    for d in np.unique(denom):
        d = int(d)
        sel = denom == d
        if d == 0:
            lut = np.zeros(1, dtype=np.float64)   # common == denom == 0 -> 0 (Mash)
        else:
            lut = _lib.distance_lut(d, k)
        txt = "\n".join("%g" % v for v in lut) + "\n"
        lut32 = pd.read_csv(io.StringIO(txt), header=None, names=['dist'],
                            dtype={'dist': np.float32}, sep='\t')['dist'].to_numpy()
        out[sel] = lut32[common[sel]]
    return out


def float32_tables(denominators, s: int, k: int = MASH_K):
    """(lut32, lut_off) for every denominator d that occurs: lut32[lut_off[d] +
    c] = the float32 "dist" of (common c, denominator d) as the reference
    parses it (mash_distance_float32); lut_off has s + 1 entries, -1 where d
    does not occur."""
    lut_off = np.full(s + 1, -1, dtype=np.int32)
    parts, pos = [], 0
    for d in np.asarray(denominators, dtype=np.int64):
        d = int(d)
        c = np.arange(d + 1, dtype=np.uint16)
        parts.append(mash_distance_float32(c, np.full(d + 1, d, dtype=np.uint16), k))
        lut_off[d] = pos
        pos += d + 1
    lut32 = np.concatenate(parts).astype(np.float32) if parts else np.zeros(1, np.float32)
    return lut32, lut_off


def _denominators(denom: np.ndarray, s: int):
    """(distinct denominators, whether every pair has denominator s) without
    sorting the condensed vector (5x10^7 entries at 10^4 genomes)."""
    denom = np.asarray(denom)
    if denom.size == 0 or (denom == s).all():
        return np.array([s]), True
    seen = np.bincount(denom.astype(np.int64, copy=False), minlength=s + 1) > 0
    return np.nonzero(seen)[0], False


def mdb_from_condensed(names: Sequence[str], common: np.ndarray, denom: np.ndarray,
                       nhash: np.ndarray, s: int, k: int = MASH_K, threads: int = 0) -> pd.DataFrame:
    """Long-form Mdb (genome1, genome2, dist, similarity) from the condensed
    all-pairs result, with the reference's row order (outer loop = query =
    genome2, inner = reference = genome1, as `mash dist` prints), dtypes
    (ordered categoricals sorted by name; float32) and values
    (d_cluster.py:575-596).

    The N^2 rows are filled by libdrephip on host threads
    (drephip_mdb_square): the float32 distances from one table per
    denominator (the reference's %g / read_csv values, float32_tables), the
    diagonal 0 -- a genome against itself has common = denom = its hash count
    (or 0 for an empty sketch), distance 0 either way --, similarity = 1 - dist
    in float32, and the category codes of both columns; the DataFrame wraps
    those arrays without copying them."""
    N = len(names)
    common = np.asarray(common, dtype=np.uint16)
    dens, full = _denominators(np.asarray(denom, dtype=np.uint16), s)
    lut32, lut_off = float32_tables(dens, s, k)
    cats = sorted(set(names))
    dtype = pd.CategoricalDtype(cats, ordered=True)
    code_t = pd.Categorical([], dtype=dtype).codes.dtype        # pandas' code width for len(cats)
    pos = {n: i for i, n in enumerate(cats)}
    codes = np.array([pos[n] for n in names], dtype=code_t)
    g1, g2, dist, sim = _lib.mdb_square(N, common, None if full else denom, s, lut32, lut_off, codes, threads)
    return pd.DataFrame({'genome1': pd.Categorical.from_codes(g1, dtype=dtype, validate=False),
                         'genome2': pd.Categorical.from_codes(g2, dtype=dtype, validate=False),
                         'dist': dist, 'similarity': sim}, copy=False)


# ---------------------------------------------------------- devices
def _devices(kwargs) -> List[int]:
    """HIP devices for the Mash step: kwargs `gpus` (a count, a list, or
    "0,1,..."), else $DREPHIP_DEVICES, else the single `gpu` /
    $DREPHIP_DEVICE (default 0)."""
    g = kwargs.get('gpus', os.environ.get('DREPHIP_DEVICES'))
    if g is None or g == '':
        return [int(kwargs.get('gpu', os.environ.get('DREPHIP_DEVICE', 0)))]
    if isinstance(g, int):
        return list(range(g))
    if isinstance(g, str):
        return [int(x) for x in g.split(',') if x.strip() != '']
    return [int(x) for x in g]


def _on_devices(devs: Sequence[int], fn) -> list:
    """fn(i, device) for every device, one host thread each (the C ABI calls
    release the GIL); first exception re-raised."""
    from concurrent.futures import ThreadPoolExecutor
    if len(devs) == 1:
        return [fn(0, devs[0])]
    with ThreadPoolExecutor(max_workers=len(devs)) as ex:
        futs = [ex.submit(fn, i, d) for i, d in enumerate(devs)]
        return [f.result() for f in futs]


def _balanced_shards(weights: Sequence[int], n: int) -> List[List[int]]:
    """Contiguous index shards with near-equal total weight (genome bytes)."""
    w = np.asarray(weights, dtype=np.float64)
    cum = np.concatenate([[0.0], np.cumsum(w)])
    cuts = [0] + [int(np.searchsorted(cum, cum[-1] * k / n)) for k in range(1, n)] + [len(w)]
    cuts = np.maximum.accumulate(np.minimum(cuts, len(w)))
    return [list(range(cuts[k], cuts[k + 1])) for k in range(n)]


# ---------------------------------------------------------- sketch cache
def _load_cached(path: str, s: int) -> Optional[MashReference]:
    try:
        m = read_msh(path)
    except Exception:
        return None
    if m.kmer != MASH_K or m.sketch_size != s or m.seed != MASH_SEED or len(m.references) != 1:
        return None
    return m.references[0]


@dataclass
class SketchSet:
    names: List[str]          # genome (basename), Bdb order
    locations: List[str]
    hashes: np.ndarray        # uint64 [N, s], rows padded with UINT64_MAX
    nhash: np.ndarray         # uint32 [N]
    length: np.ndarray        # uint64 [N]
    s: int


def sketch_genomes(Bdb: pd.DataFrame, data_folder: str, **kwargs) -> SketchSet:
    """The sketch + paste half of all_vs_all_MASH (d_cluster.py:499-567):
    same folders and files (MASH_files/sketches/chunk_<i>/<genome>.msh,
    chunk_all.msh, ALL.msh), sketches cached across runs by file existence
    (d_cluster.py:541-542), new ones computed on the GPU in one batch."""
    MASH_s = int(kwargs.get('MASH_sketch', 1000))
    p = int(kwargs.get('processors', 6))
    groupSize = int(kwargs.get('groupSize', 1000))
    write_sketches = kwargs.get('write_sketches', True)

    MASH_folder = os.path.join(data_folder, 'MASH_files/')
    sketch_folder = os.path.join(MASH_folder, 'sketches/')
    os.makedirs(sketch_folder, exist_ok=True)

    l2g = Bdb.set_index('location')['genome'].to_dict()
    locations = list(Bdb['location'].unique())
    chunks = [locations[x:x + groupSize] for x in range(0, len(locations), groupSize)]
    N = len(locations)
    names = [l2g[loc] for loc in locations]
    hashes = np.full((N, MASH_s), np.iinfo(np.uint64).max, dtype=np.uint64)
    nhash = np.zeros(N, dtype=np.uint32)
    length = np.zeros(N, dtype=np.uint64)
    msh_path: Dict[int, str] = {}
    todo: List[int] = []
    idx = 0
    chunk_members: List[List[int]] = []
    cache = _Stage('sketch_cache_s')
    cache.__enter__()
    for i, chunk in enumerate(chunks):
        chunk_folder = os.path.join(sketch_folder, "chunk_{0}".format(i))
        os.makedirs(chunk_folder, exist_ok=True)
        members = []
        for _ in chunk:
            f = os.path.join(chunk_folder, names[idx]) + '.msh'
            msh_path[idx] = f
            ref = _load_cached(f, MASH_s) if os.path.isfile(f) else None
            if ref is not None:
                n = min(len(ref.hashes), MASH_s)
                hashes[idx, :n] = ref.hashes[:n]
                nhash[idx] = n
                length[idx] = ref.length
            else:
                todo.append(idx)
            members.append(idx)
            idx += 1
        chunk_members.append(members)
    cache.__exit__()
    STAGE_TIMES['sketched_genomes'] = len(todo)

    sk = _Stage('sketch_gpu_s')
    sk.__enter__()
    if todo:
        devs = _devices(kwargs)
        sizes = [os.path.getsize(locations[i]) if os.path.exists(locations[i]) else 1 for i in todo]
        shards = [[todo[j] for j in sh] for sh in _balanced_shards(sizes, len(devs))]
        threads = max(1, p // len(devs))

        def run(k, dev):
            if not shards[k]:
                return
            with _lib.Context(device=dev, k=MASH_K, s=MASH_s, seed=MASH_SEED) as ctx:
                h, nh, ln = ctx.sketch_files([locations[i] for i in shards[k]], threads=threads)
            hashes[shards[k]] = h
            nhash[shards[k]] = nh
            length[shards[k]] = ln
        _on_devices(devs, run)
        logging.debug("sketched %d genomes on HIP devices %s", len(todo), devs)
    sk.__exit__()

    wr = _Stage('sketch_write_s')
    wr.__enter__()
    if write_sketches:
        def ref_of(i):
            return MashReference(locations[i], '', int(length[i]), hashes[i, :nhash[i]])
        for i in todo:
            write_msh(msh_path[i], [ref_of(i)], MASH_K, MASH_s, MASH_SEED)
        alls = []
        for ci, members in enumerate(chunk_members):
            all_file = os.path.join(sketch_folder, "chunk_{0}".format(ci), 'chunk_all.msh')
            write_msh(all_file, [ref_of(i) for i in members], MASH_K, MASH_s, MASH_SEED)
            alls.append(all_file)
        write_msh(os.path.join(MASH_folder, 'ALL.msh'), [ref_of(i) for i in range(N)],
                  MASH_K, MASH_s, MASH_SEED)
    wr.__exit__()
    return SketchSet(names, locations, hashes, nhash, length, MASH_s)


@dataclass
class CondensedMash:
    names: List[str]
    locations: List[str]
    common: np.ndarray     # uint16, condensed i<j (scipy squareform order)
    denom: np.ndarray      # uint16, same layout
    nhash: np.ndarray
    length: np.ndarray
    s: int


def all_vs_all_MASH_condensed(Bdb, data_folder, **kwargs) -> CondensedMash:
    """Sketch (or load cached sketches) and run the HIP all-pairs kernel;
    return the condensed shared-hash counts instead of an N^2-row table."""
    sk = sketch_genomes(Bdb, data_folder, **kwargs)
    with _Stage('allpairs_s'):
        common, denom = condensed_allpairs(sk.hashes, sk.nhash, sk.s, _devices(kwargs))
    return CondensedMash(sk.names, sk.locations, common, denom, sk.nhash, sk.length, sk.s)


def condensed_allpairs(hashes: np.ndarray, nhash: np.ndarray, s: int, devices: Sequence[int] = (0,)):
    """(common, denom) for the whole condensed triangle.  With several devices
    the rows are split into contiguous ranges of near-equal pair count
    (parallel.row_partition), one context and host thread per device, each
    writing its own segment of the host buffers (no collective)."""
    N = len(nhash)
    npairs = N * (N - 1) // 2
    partial = bool((np.asarray(nhash) < s).any())
    common = np.zeros(npairs, dtype=np.uint16)
    denom = np.zeros(npairs, dtype=np.uint16) if partial else None
    parts = row_partition(N, len(devices))

    def run(k, dev):
        r0, r1 = parts[k]
        a = cond_start(r0, N)
        b = a + segment_size(N, r0, r1)
        if b <= a:
            return
        with _lib.Context(device=dev, k=MASH_K, s=s, seed=MASH_SEED) as ctx:
            ctx.allpairs_rows(hashes, nhash, r0, r1, common[a:b], denom[a:b] if denom is not None else None)
    if npairs:
        _on_devices(list(devices), run)
    if denom is None:
        denom = np.full(npairs, s, dtype=np.uint16)
    return common, denom


def all_vs_all_MASH(Bdb, data_folder, **kwargs):
    """
    Run MASH pairwise within all samples in Bdb (reference
    drep/d_cluster.py:481-596), with sketching and the all-vs-all distance on
    the GPU.

    Args:
        Bdb: dataframe with genome, location
        data_folder: location to store output files

    Keyword Args:
        MASH_sketch: size of mash sketches (int or str, as the CLI passes it)
        dry: dont actually run anything (parses an existing MASH_table.tsv, as
            the reference does after printing its commands)
        processors: CPU threads for FASTA ingest
        groupSize: max number of mash sketches to hold in each folder
        debug / wd: accepted for compatibility (no external commands to log)
        exe_loc / mash_exe: accepted and ignored (no mash executable is used)
        gpu: HIP device index (default $DREPHIP_DEVICE or 0)
        gpus: several HIP devices (count, list or "0,1,..."; default
            $DREPHIP_DEVICES): sketch shards and all-pairs row ranges run on
            all of them from this process, one host thread per device
        write_sketches: write the .msh files (default True)
        write_table: also write MASH_table.tsv like `mash dist` (default False)

    Returns:
        Mdb DataFrame [genome1, genome2, dist, similarity]
    """
    MASH_folder = os.path.join(data_folder, 'MASH_files/')
    if kwargs.get('dry', False):
        table = MASH_folder + 'MASH_table.tsv'
        print("# drep_amd: dry run -- would sketch %d genomes and run all-pairs on HIP device %s"
              % (len(Bdb), kwargs.get('gpu', os.environ.get('DREPHIP_DEVICE', 0))))
        return _parse_mash_table(table, Bdb)

    STAGE_TIMES.clear()
    cm = all_vs_all_MASH_condensed(Bdb, data_folder, **kwargs)
    if kwargs.get('write_table', False):
        with _Stage('mash_table_s'):
            write_mash_table(MASH_folder + 'MASH_table.tsv', cm)
    with _Stage('mdb_s'):
        Mdb = mdb_from_condensed(cm.names, cm.common, cm.denom, cm.nhash, cm.s,
                                 threads=int(kwargs.get('processors', 6)))

    # Filter out those genomes that are not in Bdb (reference 586-594).  When
    # every sketched genome is in Bdb (the drop-in sketches Bdb's own genomes)
    # the block is the identity: no row is dropped and the categories already
    # are the sorted names, ordered (mdb_from_condensed) -- skip its 10^6-row
    # isin passes
    genomes = Bdb['genome'].unique()
    if set(cm.names).issubset(set(genomes)):
        return Mdb
    Mdb = Mdb[Mdb['genome1'].isin(genomes)]
    Mdb = Mdb[Mdb['genome2'].isin(genomes)]
    for g in ['genome1', 'genome2']:
        Mdb[g] = Mdb[g].cat.remove_unused_categories()
        Mdb[g] = Mdb[g].cat.reorder_categories(sorted((Mdb[g].unique())), ordered=True)
    return Mdb


def _parse_mash_table(file, Bdb):
    """The reference's TSV -> Mdb parse (d_cluster.py:575-596)."""
    iniCols = ['genome1', 'genome2', 'dist', 'p', 'kmers']
    uCols = ['genome1', 'genome2', 'dist']
    dTypes = {'genome1': 'category', 'genome2': 'category', 'dist': np.float32}
    Mdb = pd.read_csv(file, names=iniCols, usecols=uCols, dtype=dTypes, sep='\t')
    Mdb['genome1'] = Mdb['genome1'].apply(_get_genome_name_from_fasta)
    Mdb['genome2'] = Mdb['genome2'].apply(_get_genome_name_from_fasta)
    Mdb['similarity'] = 1 - Mdb['dist']
    genomes = Bdb['genome'].unique()
    Mdb = Mdb[Mdb['genome1'].isin(genomes)]
    Mdb = Mdb[Mdb['genome2'].isin(genomes)]
    for g in ['genome1', 'genome2']:
        Mdb[g] = Mdb[g].astype('category').cat.remove_unused_categories()
        Mdb[g] = Mdb[g].cat.reorder_categories(sorted((Mdb[g].unique())), ordered=True)
    return Mdb


def mash_pvalue(common: np.ndarray, len_r: np.ndarray, len_q: np.ndarray, s: int,
                k: int = MASH_K) -> np.ndarray:
    """Mash's p-value column (binomial upper tail; Mash uses GSL's
    gsl_cdf_binomial_Q, restated with scipy): 1 if common == 0, else
    Q(common-1; r, trunc(min(M, s)))."""
    from scipy.stats import binom
    kspace = 4.0 ** k
    px = 1.0 / (1.0 + kspace / np.asarray(len_r, dtype=np.float64))
    py = 1.0 / (1.0 + kspace / np.asarray(len_q, dtype=np.float64))
    r = px * py / (px + py - px * py)
    M = kspace * (px + py) / (1.0 + r)
    n = np.floor(np.minimum(M, s))
    c = np.asarray(common, dtype=np.float64)
    p = binom.sf(c - 1, n, r)
    return np.where(c == 0, 1.0, p)


def write_mash_table(path: str, cm: CondensedMash, threads: int = 0) -> None:
    """MASH_table.tsv as `mash dist ALL ALL` prints it (d_cluster.py:570-572):
    reference, query, %g distance, %g p-value, common/denom; outer loop over
    queries.  N^2 lines (10^8 at 10^4 genomes).  Distances (per-denominator
    tables) and p-values are computed once per unordered pair -- both are
    symmetric in (reference, query) -- and only for pairs sharing a hash (the
    p-value of c = 0 is 1); libdrephip formats the text on `threads` host
    threads (drephip_write_mash_table)."""
    N = len(cm.names)
    common = np.asarray(cm.common, dtype=np.uint16)
    denom = np.asarray(cm.denom, dtype=np.uint16)
    length = np.asarray(cm.length, dtype=np.float64)
    dist = np.empty(len(common), dtype=np.float64)
    for d in np.unique(denom):
        sel = denom == d
        lut = _lib.distance_lut(int(d), MASH_K) if d else np.zeros(1)
        dist[sel] = lut[common[sel]]
    pval = np.ones(len(common), dtype=np.float64)
    nz = np.nonzero(common)[0]
    if len(nz):
        iu, ju = _condensed_ij(nz, N)
        pval[nz] = mash_pvalue(common[nz], length[iu], length[ju], cm.s)
    self_count = np.minimum(np.asarray(cm.nhash, dtype=np.int64), cm.s).astype(np.uint16)
    self_pval = mash_pvalue(self_count, length, length, cm.s)
    full = bool((denom == cm.s).all())
    _lib.write_mash_table(path, list(cm.locations), common, None if full else denom, cm.s, dist, pval,
                          self_count, self_pval, threads)


def _condensed_ij(t: np.ndarray, N: int):
    """(i, j), i < j, of condensed indices t (scipy squareform order)."""
    t = np.asarray(t, dtype=np.int64)
    Mf = 2.0 * N - 1.0
    i = np.floor((Mf - np.sqrt(np.maximum(Mf * Mf - 8.0 * t, 0.0))) / 2.0).astype(np.int64)
    i = np.clip(i, 0, max(N - 2, 0))
    for _ in range(2):
        i = np.where(i * N - i * (i + 1) // 2 > t, i - 1, i)
        i = np.where((i + 1) * N - (i + 1) * (i + 2) // 2 <= t, i + 1, i)
    j = t - (i * N - i * (i + 1) // 2) + i + 1
    return i, j


# ------------------------------------------------------ primary clustering
def _primary_cdb(labels, names) -> pd.DataFrame:
    """Cdb [primary_cluster, genome]: fcluster labels in the pivot's genome
    order (what dRep's _gen_cdb_from_fclust + rename give,
    d_cluster.py:463-479, 623)."""
    return pd.DataFrame({'primary_cluster': np.asarray(labels), 'genome': list(names)})


def _pivot_dist(db: pd.DataFrame) -> pd.DataFrame:
    """db.pivot(index="genome1", columns="genome2", values="dist")
    (d_cluster.py:620; keyword form -- pandas >= 2 rejects the positional one),
    the same DataFrame, filled by libdrephip on category codes
    (drephip_pivot_scan / drephip_pivot_fill) when the table is what the
    Mash step produces: both genome columns categorical over one sorted list
    of names (the reference's parse sorts them, d_cluster.py:591-594) and a
    float32 dist.  Index and columns are then the names that occur, in
    category order, as CategoricalIndex of the column's dtype (pandas' pivot of
    a categorical); missing cells NaN; a cell named twice raises pandas'
    ValueError.  Any other table goes through pandas itself."""
    g1, g2, dist = db['genome1'], db['genome2'], db['dist']
    fast = (isinstance(g1.dtype, pd.CategoricalDtype) and isinstance(g2.dtype, pd.CategoricalDtype)
            and g1.dtype.categories.equals(g2.dtype.categories) and g1.dtype.ordered == g2.dtype.ordered
            and g1.dtype.categories.is_monotonic_increasing and dist.dtype == np.float32 and len(db) > 0)
    if fast:
        c1 = g1.cat.codes.to_numpy()
        c2 = g2.cat.codes.to_numpy()
        fast = c1.dtype == c2.dtype and c1.dtype in (np.int8, np.int16, np.int32)
    if not fast:
        return db.pivot(index="genome1", columns="genome2", values="dist")
    ncat = len(g1.dtype.categories)
    try:
        p1, p2, period = _lib.pivot_scan(c1, c2, ncat)
    except _lib.DrepHipError:                   # a missing genome (NaN category): pandas' own handling
        return db.pivot(index="genome1", columns="genome2", values="dist")
    if not (p1.all() and p2.all()):
        # a category unused in either column: pandas' unstack then orders the
        # names in a way of its own (not the category order) -- leave it to pandas
        return db.pivot(index="genome1", columns="genome2", values="dist")
    pos1 = np.where(p1, np.cumsum(p1) - 1, -1).astype(np.int32)
    pos2 = np.where(p2, np.cumsum(p2) - 1, -1).astype(np.int32)
    n1, n2 = int(p1.sum()), int(p2.sum())
    try:
        M = _lib.pivot_fill(c1, c2, pos1, pos2, dist.to_numpy(), n1, n2, period)
    except _lib.DrepHipError as e:
        raise ValueError("Index contains duplicate entries, cannot reshape") from e

    def index(present, name, dtype):
        return pd.CategoricalIndex(pd.Categorical.from_codes(np.nonzero(present)[0], dtype=dtype), name=name)
    return pd.DataFrame(M, index=index(p1, "genome1", g1.dtype), columns=index(p2, "genome2", g2.dtype), copy=False)


def _linkage_gpu(kwargs) -> Optional[int]:
    """The HIP device of the primary linkage: kwargs `gpu` (None = scipy on
    the host), else $DREPHIP_DEVICE, else 0."""
    if 'gpu' in kwargs:
        return None if kwargs['gpu'] is None else int(kwargs['gpu'])
    return int(os.environ.get('DREPHIP_DEVICE', 0))


def _square_linkage(M: np.ndarray, method: str, gpu: int) -> np.ndarray:
    """scipy.cluster.hierarchy.linkage(squareform(M), method) on the GPU (Z
    bit-identical): float32 M through drephip_linkage_square (squareform's and
    linkage's checks on the device), float64 M through squareform +
    drephip_linkage.  A failed check raises scipy's ValueError."""
    with _lib.Context(device=gpu, k=MASH_K, s=1, seed=MASH_SEED) as ctx:
        if M.dtype == np.float32:
            try:
                return ctx.linkage_square(M, method)
            except _lib.DrepHipError as e:
                msg = _lib.lib().drephip_last_error().decode("utf-8", "replace")
                if msg in ("Distance matrix 'X' must be symmetric.", "Distance matrix 'X' diagonal must be zero.",
                           "The condensed distance matrix must contain only finite values."):
                    raise ValueError(msg) from e
                raise
        y = ssd.squareform(np.asarray(M, dtype=np.float64))
        if not np.all(np.isfinite(y)):
            raise ValueError("The condensed distance matrix must contain only finite values.")
        return ctx.linkage(y, method)


def cluster_mash_database(db, **kwargs):
    """
    From a Mash database, cluster and return Cdb (reference
    drep/d_cluster.py:598-630, with its cluster_hierarchical 429-461).  Same
    in-place update of db['dist'] from db['similarity'] as the reference, the
    same pivot (pandas' DataFrame, filled from the category codes by
    libdrephip: _pivot_dist) and the same linkage of its squareform -- run on
    the GPU for single / complete / average / weighted (scipy's algorithms
    restated, Z bit-identical; drephip_linkage_square), by scipy for the other
    methods -- so Cdb, linkage and linkage_db equal the reference's.

    Keyword arguments:
        clusterAlg: how to cluster database (default = single)
        P_ani: threshold to cluster at (default = 0.9)
        gpu: HIP device of the linkage (default $DREPHIP_DEVICE or 0); None
            runs scipy's linkage on the host, as the reference does

    Returns:
        list: [Cdb, [linkage, linkage_db, arguments]]
    """
    logging.debug('Clustering MASH database')
    method = kwargs.get('clusterAlg', 'single')
    cutoff = 1 - kwargs.get('P_ani', .9)
    with _Stage('dist_update_s'):
        db['dist'] = 1 - db['similarity']
    with _Stage('pivot_s'):
        linkage_db = _pivot_dist(db)
    gpu = _linkage_gpu(kwargs)
    M = np.asarray(linkage_db)
    link = _Stage('linkage_s')
    link.__enter__()
    try:
        if (gpu is not None and method in GPU_LINKAGE_METHODS and M.ndim == 2 and M.shape[0] == M.shape[1]
                and M.shape[0] >= 2 and M.dtype in (np.float32, np.float64)):
            linkage = _square_linkage(M, method, gpu)
        else:
            y = ssd.squareform(M)       # raises unless symmetric with a zero diagonal
            linkage = scipy.cluster.hierarchy.linkage(y, method=method)
    except ValueError as e:
        if "symmetric" in str(e) or "diagonal" in str(e) or "square" in str(e):    # squareform's checks
            logging.error("The database passed in is not symmetrical!")
        raise
    link.__exit__()
    labels = scipy.cluster.hierarchy.fcluster(linkage, cutoff, criterion='distance')
    Cdb = _primary_cdb(labels, linkage_db.columns)
    arguments = {'linkage_method': method, 'linkage_cutoff': cutoff, 'comparison_algorithm': 'MASH'}
    return Cdb, [linkage, linkage_db, arguments]


def _linkage_values(common: np.ndarray, denom: np.ndarray) -> np.ndarray:
    """float64 linkage input for (common, denom) pairs, bit-identical to what
    the reference feeds scipy: dist32 (the %g / read_csv path) -> 1 - (1 -
    dist32) in float32 (d_cluster.py:584, 619) -> float64."""
    d32 = mash_distance_float32(common, denom)
    one = np.float32(1)
    return (one - (one - d32)).astype(np.float32).astype(np.float64)


def condensed_cluster_distances(cm: CondensedMash) -> np.ndarray:
    """float64 condensed linkage input, rows/columns in sorted-name order (the
    pivot's order)."""
    N = len(cm.names)
    after = _linkage_values(cm.common, cm.denom)
    order = np.argsort(np.array(cm.names, dtype=object), kind='stable')
    if np.all(order == np.arange(N)):
        return after
    M = ssd.squareform(after, checks=False)[np.ix_(order, order)]
    return ssd.squareform(M, checks=False).astype(np.float64)


def linkage_tables(denominators: np.ndarray, s: int):
    """(lut, lut_off) for drephip_linkage_counts_device: for every denominator
    d that occurs, lut[lut_off[d] + c] = linkage input value of (c, d)."""
    lut_off = np.full(s + 1, -1, dtype=np.int32)
    parts, pos = [], 0
    for d in np.unique(np.asarray(denominators)):
        d = int(d)
        c = np.arange(d + 1)
        parts.append(_linkage_values(c, np.full(d + 1, d)))
        lut_off[d] = pos
        pos += d + 1
    lut = np.concatenate(parts) if parts else np.zeros(1)
    return lut, lut_off


def linkage_order(names: Sequence[str]) -> np.ndarray:
    """perm[i] = row of genome i in the linkage input (sorted names, as the
    reference's pivot orders them)."""
    order = np.argsort(np.array(names, dtype=object), kind='stable')
    perm = np.empty(len(names), dtype=np.uint32)
    perm[order] = np.arange(len(names), dtype=np.uint32)
    return perm


GPU_LINKAGE_METHODS = ('single', 'complete', 'average', 'weighted')


def cluster_mash_condensed(cm: CondensedMash, **kwargs):
    """Primary clustering straight from the condensed result (no N^2 Mdb):
    same linkage input as cluster_mash_database builds via pivot+squareform.

    The linkage runs on the GPU (libdrephip drephip_linkage_counts_device:
    scipy's nn_chain / MST restated, Z bit-identical; the n x n matrix is
    built in HBM from the counts) on device `gpu` (default $DREPHIP_DEVICE or
    0); other methods, or gpu=None, use scipy on the host."""
    P_Lmethod = kwargs.get('clusterAlg', 'single')
    P_Lcutoff = 1 - kwargs.get('P_ani', .9)
    gpu = _linkage_gpu(kwargs)
    names = sorted(cm.names)
    N = len(cm.names)
    if gpu is not None and P_Lmethod in GPU_LINKAGE_METHODS and N >= 2:
        import torch
        dev = torch.device('cuda', int(gpu))
        lut, lut_off = linkage_tables(cm.denom, cm.s)
        d_c = torch.from_numpy(np.ascontiguousarray(cm.common, dtype=np.uint16).view(np.int16)).to(dev)
        full = bool((cm.denom == cm.s).all())
        d_d = None if full else torch.from_numpy(np.ascontiguousarray(cm.denom, dtype=np.uint16).view(np.int16)).to(dev)
        torch.cuda.synchronize(dev)
        with _lib.Context(device=int(gpu), k=MASH_K, s=cm.s, seed=MASH_SEED) as ctx:
            linkage = ctx.linkage_counts_device(d_c.data_ptr(), None if d_d is None else d_d.data_ptr(), N,
                                                linkage_order(cm.names), lut, lut_off, P_Lmethod)
    else:
        arr = condensed_cluster_distances(cm)
        linkage = scipy.cluster.hierarchy.linkage(arr, method=P_Lmethod)
    fclust = scipy.cluster.hierarchy.fcluster(linkage, P_Lcutoff, criterion='distance')
    Cdb = _primary_cdb(fclust, names)
    arguments = {'linkage_method': P_Lmethod, 'linkage_cutoff': P_Lcutoff,
                 'comparison_algorithm': 'MASH'}
    return Cdb, [linkage, None, arguments]
