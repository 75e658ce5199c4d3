"""Sharded Mash step + primary clustering across the GPUs of one node
(BASELINE configs[3]: 10^5 genomes on 8 x MI355X).  One process per GPU
(torchrun), RCCL over xGMI through torch.distributed ("nccl" backend); gloo
on CPU in the tests.

The reference does all of this in one process: `mash sketch` per genome on a
thread pool, `mash paste`, `mash dist -p P` into one TSV, then scipy linkage
on the pivoted Mdb (drep/d_cluster.py:170-185 -> all_vs_all_MASH 481-596 ->
cluster_mash_database 598-630 -> store_special('primary_linkage')).  Here:

  1. sketch      rank r sketches its contiguous genome shard (HIP kernels)
  2. exchange    ONE all-gather of the uint64[N/W][s] sketch shards (+ counts)
  3. all-pairs   rank r computes the rows [r0, r1) of the triangle balanced by
                 pair count (parallel.row_partition): one contiguous condensed
                 segment per rank
  4. gather      every segment goes to the root GPU, straight into its slice
                 of one condensed buffer: point-to-point send/recv (the
                 segments are uneven, so no padded collective), all receives
                 posted at once so the 7 xGMI links run in parallel
  5. clustering  on the root GPU: the n x n linkage input built in HBM from
                 the counts, scipy's linkage algorithm restated (Z
                 bit-identical, libdrephip drephip_linkage_counts_device),
                 fcluster -> Cdb; optionally stored in the work-directory
                 formats of drep_amd.store (condensed counts + the reference's
                 primary_linkage pickle).

The stage functions are parameters of run_sharded so the plumbing (shards,
gather order, uneven segments, root assembly) is the same code whether the
per-rank compute is the HIP library (product) or a CPU stand-in (the gloo
tests in tests/test_parallel.py).
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .parallel import (balanced_shards, cond_start, gather_sketches, genome_shard, row_partition, segment_size,
                       shard_layout)


@dataclass
class ShardPlan:
    N: int
    world: int
    rank: int
    g0: int          # contiguous shards: this rank's genomes [g0, g1) (balanced shards: -1)
    g1: int
    nmax: int        # padded shard size (every rank's all-gather chunk)
    r0: int          # this rank's triangle rows [r0, r1)
    r1: int
    seg0: int        # condensed index of the segment's first pair
    seg_len: int
    members: Optional[np.ndarray] = None    # this rank's genome indices, ascending (= arange(g0, g1) if contiguous)
    pos: Optional[np.ndarray] = None        # balanced shards: gathered row of every genome (None: identity)

    def genomes(self) -> np.ndarray:
        return self.members if self.members is not None else np.arange(self.g0, self.g1)


def plan(N: int, world: int, rank: int, weights: Optional[Sequence[float]] = None) -> ShardPlan:
    """This rank's share of the job.  Without weights the genome shards are
    contiguous and of equal count (synthetic genomes of one length); with
    weights (the FASTA inputs' sizes) they are balanced by weight
    (parallel.balanced_shards) and padded to the largest shard for the
    all-gather, whose rows run_sharded then puts back in genome order."""
    r0, r1 = row_partition(N, world)[rank]
    if weights is None:
        g0, g1, nmax = genome_shard(N, world, rank)
        return ShardPlan(N, world, rank, g0, g1, nmax, r0, r1, cond_start(r0, N), segment_size(N, r0, r1),
                         members=np.arange(g0, g1))
    shards = balanced_shards(weights, world)
    nmax, pos = shard_layout(shards, N)
    return ShardPlan(N, world, rank, -1, -1, nmax, r0, r1, cond_start(r0, N), segment_size(N, r0, r1),
                     members=shards[rank], pos=pos)


def gather_segments(seg, N: int, root: int = 0, out=None):
    """Condensed segments of every rank -> one condensed vector on the root.

    seg: this rank's segment (1-D tensor; int16 views of the uint16 counts),
    on the rank's GPU with the nccl backend, on the CPU with gloo.  Returns
    the full N(N-1)/2 tensor on the root (written into `out` if given), None
    elsewhere.  Every rank takes part in one batch_isend_irecv: the root posts
    a receive per other rank into that rank's slice, the others one send."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    parts = row_partition(N, world)
    sizes = [segment_size(N, a, b) for a, b in parts]
    if seg.numel() < sizes[rank]:
        raise ValueError("rank %d segment has %d pairs, expected %d" % (rank, seg.numel(), sizes[rank]))
    # gloo moves host memory only: device segments are staged through the host
    # (rehearsals of the sharded path on one GPU; RCCL moves device memory)
    host_p2p = dist.get_backend() == "gloo" and seg.is_cuda
    # the transfers move bytes (int8 views): NCCL/RCCL has no 16-bit integer
    # type, and torch's nccl process group rejects int16 tensors
    def as_bytes(t):
        return t.view(torch.int8)
    ops, landing = [], []
    full = None
    if rank == root:
        npairs = N * (N - 1) // 2
        full = out if out is not None else torch.empty(npairs, dtype=seg.dtype, device=seg.device)
        if full.numel() != npairs:
            raise ValueError("output holds %d pairs, expected %d" % (full.numel(), npairs))
        for r, (a, b) in enumerate(parts):
            if not sizes[r]:
                continue
            lo = cond_start(a, N)
            if r == root:
                if seg.data_ptr() != full[lo:lo + sizes[r]].data_ptr():   # not already in place
                    full[lo:lo + sizes[r]].copy_(seg[:sizes[r]])
            elif host_p2p:
                buf = torch.empty(sizes[r], dtype=seg.dtype)
                landing.append((full[lo:lo + sizes[r]], buf))
                ops.append(dist.P2POp(dist.irecv, as_bytes(buf), r))
            else:
                ops.append(dist.P2POp(dist.irecv, as_bytes(full[lo:lo + sizes[r]]), r))
    elif sizes[rank]:
        mine = seg[:sizes[rank]].contiguous()
        ops.append(dist.P2POp(dist.isend, as_bytes(mine.cpu() if host_p2p else mine), root))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for dst, buf in landing:
        dst.copy_(buf)
    return full


POISON = -1            # int16 view of 0xFFFF: an impossible shared-hash count (s <= 32767)

SketchFn = Callable[[ShardPlan], Tuple["object", "object"]]            # -> (loc_h [nmax, s], loc_n [nmax])
AllpairsFn = Callable[..., Tuple["object", Optional["object"]]]      # fn(H, NH, plan, out=None)
LinkageFn = Callable[["object", Optional["object"], int, str], np.ndarray]


def run_sharded(N: int, names: Sequence[str], s: int, sketch_fn: SketchFn, allpairs_fn: AllpairsFn,
                linkage_fn: LinkageFn, method: str = "average", P_ani: float = 0.9, root: int = 0,
                sync: Optional[Callable[[], None]] = None, weights: Optional[Sequence[float]] = None) -> Dict:
    """The sharded pipeline on this rank (torch.distributed initialised).

    Returns, on the root, {'Cdb', 'linkage', 'arguments', 'common', 'denom',
    'hashes', 'nhash', 'times'}; on the other ranks {'times'}.  `sync` waits
    for this rank's device work (torch.cuda.synchronize on GPU ranks) so the
    stage times are real.  `weights` (per genome, e.g. FASTA sizes) balances
    the sketch shards by work instead of by count (plan())."""
    import torch
    import torch.distributed as dist
    import scipy.cluster.hierarchy as sch
    from .d_cluster import _primary_cdb
    world, rank = dist.get_world_size(), dist.get_rank()
    p = plan(N, world, rank, weights)
    sync = sync or (lambda: None)
    times: Dict[str, float] = {}

    def stage(name, fn):
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        out = fn()
        sync()
        dist.barrier()
        times[name] = time.perf_counter() - t0
        return out

    loc_h, loc_n = stage("sketch_s", lambda: sketch_fn(p))
    H, NH = stage("allgather_s", lambda: gather_sketches(loc_h, loc_n))
    if p.pos is None:
        H, NH = H[:N], NH[:N]
    else:                                    # balanced shards: gathered rows back to genome order
        idx = torch.from_numpy(p.pos).to(H.device)
        H, NH = H[idx].contiguous(), NH[idx].contiguous()
    partial = bool((NH < s).any().item()) if N else False
    # the root's rows are written straight into its slice of the full condensed
    # vector, so gathering the segments copies nothing on the root (at 10^5
    # genomes on one GPU that was a 10 GB device copy plus its allocation)
    full_c = None
    out = None
    # DREPHIP_SEGMENT_POISON=1 (tests): the root's vector starts as POISON, a
    # value no count takes (s <= 32767), and no pair may still hold it after the
    # gather -- every kernel path must write every pair of its rows
    poison = os.environ.get("DREPHIP_SEGMENT_POISON") == "1"
    if rank == root and N >= 2:
        npairs = N * (N - 1) // 2
        full_c = (torch.full((npairs,), POISON, dtype=torch.int16, device=H.device) if poison
                  else torch.empty(npairs, dtype=torch.int16, device=H.device))
        lo = cond_start(p.r0, N)
        out = full_c[lo:lo + p.seg_len]
    seg_c, seg_d = stage("allpairs_s", lambda: allpairs_fn(H, NH, p, out=out))
    full_c = stage("gather_segments_s", lambda: gather_segments(seg_c, N, root, out=full_c))
    if poison and full_c is not None:
        left = int((full_c == POISON).sum().item())
        if left:
            raise RuntimeError("%d pairs of the condensed vector were never written" % left)
    full_d = None
    if partial:
        if seg_d is None:
            raise ValueError("partial sketches need the denominators")
        full_d = stage("gather_denominators_s", lambda: gather_segments(seg_d, N, root))
    res: Dict = {"times": times, "plan": p}
    if rank == root:
        t0 = time.perf_counter()
        Z = linkage_fn(full_c, full_d, N, method)
        sync()
        times["linkage_s"] = time.perf_counter() - t0
        cutoff = 1 - P_ani
        fcl = sch.fcluster(Z, cutoff, criterion="distance")
        Cdb = _primary_cdb(fcl, sorted(names))
        res.update(Cdb=Cdb, linkage=Z, common=full_c, denom=full_d, hashes=H, nhash=NH,
                   arguments={"linkage_method": method, "linkage_cutoff": cutoff, "comparison_algorithm": "MASH"})
    return res


# ------------------------------------------------------------ HIP stages
def hip_synth_sketcher(ctx, L: int, family_size: int, seed: int, stream: int, device):
    """Stage 1 for synthetic genomes (the configs' workload): this rank's shard
    generated in HBM by the bench generator and sketched, CH genomes at a
    time (the packed input of 10^4 genomes is ~19 GB)."""
    import torch
    from . import _lib

    def fn(p: ShardPlan):
        s = ctx.s
        loc_h = torch.full((p.nmax, s), -1, dtype=torch.int64, device=device)
        loc_n = torch.zeros(p.nmax, dtype=torch.int32, device=device)
        n = p.g1 - p.g0
        if n <= 0:
            return loc_h, loc_n
        CH = min(n, 10_000)
        tile = _lib.tile_bases()
        P = _lib.padded_bases([L])
        codes = torch.zeros((tile + CH * P) // 16, dtype=torch.int32, device=device)
        valid = torch.zeros((tile + CH * P) // 32, dtype=torch.int32, device=device)
        for a in range(0, n, CH):
            m = min(CH, n - a)
            ctx.synth_device(seed, p.g0 + a, m, family_size, L, codes.data_ptr(), valid.data_ptr(), stream)
            ctx.sketch_device(codes.data_ptr(), valid.data_ptr(), np.array([tile + i * P for i in range(m)], np.uint64),
                              np.full(m, P, np.uint64), np.full(m, L - 20, np.uint64), m,
                              loc_h[a].data_ptr(), loc_n[a:].data_ptr(), stream)
        del codes, valid
        return loc_h, loc_n
    return fn


def hip_file_sketcher(ctx, paths: Sequence[str], threads: int, device, cached: Optional[Dict[int, object]] = None,
                      lengths: Optional[np.ndarray] = None):
    """Stage 1 for FASTA files (the files dRep passes, d_cluster.py:527-549):
    this rank's shard of the files read, packed and sketched
    (drephip_sketch_files), then moved to the rank's GPU.  `cached` maps a
    genome index to the MashReference of its existing .msh sketch (dRep's
    file-existence cache, d_cluster.py:541-542): those are not read at all.
    Genome lengths (the .msh length field) go to `lengths` when given."""
    import torch
    cached = cached or {}

    def fn(p: ShardPlan):
        s = ctx.s
        loc_h = torch.full((p.nmax, s), -1, dtype=torch.int64, device=device)
        loc_n = torch.zeros(p.nmax, dtype=torch.int32, device=device)
        mine = p.genomes()
        n = len(mine)
        if n <= 0:
            return loc_h, loc_n
        h = np.full((n, s), np.iinfo(np.uint64).max, dtype=np.uint64)
        nh = np.zeros(n, dtype=np.uint32)
        ln = np.zeros(n, dtype=np.uint64)
        todo = [i for i in range(n) if int(mine[i]) not in cached]
        for i in range(n):
            ref = cached.get(int(mine[i]))
            if ref is not None:
                m = min(len(ref.hashes), s)
                h[i, :m] = ref.hashes[:m]
                nh[i] = m
                ln[i] = ref.length
        if todo:
            th, tnh, tln = ctx.sketch_files([paths[int(mine[i])] for i in todo], threads=threads)
            h[todo], nh[todo], ln[todo] = th, tnh, tln
        if lengths is not None:
            lengths[mine] = ln
        loc_h[:n] = torch.from_numpy(h.view(np.int64)).to(device)
        loc_n[:n] = torch.from_numpy(nh.view(np.int32)).to(device)
        return loc_h, loc_n
    return fn


def read_genome_list(bdb: Optional[str] = None, files: Optional[str] = None) -> Tuple[List[str], List[str]]:
    """(names, locations) of the genomes to compare: a dRep Bdb table (CSV with
    `genome` and `location` columns, data_tables/Bdb.csv) or a text file of
    FASTA paths, one per line (names = basenames, as dRep's load_genomes /
    _get_genome_name_from_fasta give them).  Locations keep Bdb's order,
    duplicates dropped (d_cluster.py:527)."""
    from .d_cluster import _get_genome_name_from_fasta
    if bdb:
        import pandas as pd
        B = pd.read_csv(bdb)
        l2g = B.set_index('location')['genome'].to_dict()
        locs = list(B['location'].unique())
        return [l2g[x] for x in locs], locs
    locs: List[str] = []
    for line in open(files):
        line = line.strip()
        if line and line not in locs:
            locs.append(line)
    return [_get_genome_name_from_fasta(x) for x in locs], locs


# uncompressed / compressed size of a gzip'd FASTA whose trailer does not tell
# (bgzip / multi-member files): nucleotide text deflates about 3.5x
GZIP_DNA_RATIO = 3.5


def gzip_bases_estimate(path: str, size: int) -> float:
    """Uncompressed size of a gzip file without inflating it.  The trailer's
    ISIZE is the LAST member's size mod 2^32: exact for the usual
    single-member file, but 0 for bgzip (BGZF ends with an empty member) and
    too small for other multi-member files or files over 4 GiB.  A BGZF header
    (FEXTRA with a 'BC' subfield), or an ISIZE below the compressed size
    (nucleotide text always deflates), falls back to size x GZIP_DNA_RATIO;
    the result is an estimate for balancing, never a length."""
    with open(path, "rb") as f:
        head = f.read(18)
        f.seek(-4, os.SEEK_END)
        isize = int.from_bytes(f.read(4), "little")
    bgzf = len(head) >= 16 and head[:2] == b"\x1f\x8b" and head[3] & 4 and head[12:14] == b"BC"
    if bgzf or isize < size:
        return float(size) * GZIP_DNA_RATIO
    return float(isize)


def file_weights(locations: Sequence[str], cached: Optional[Dict[int, object]] = None) -> np.ndarray:
    """Sketch work per genome for balanced_shards: the FASTA's bases as far as
    they are known without reading it -- the file size, or for a gzip file
    gzip_bases_estimate -- and 0 for a genome whose sketch is cached.  In a
    sharded job only the root calls it and broadcasts the result
    (main()): every rank's shard plan must come from the same weights."""
    cached = cached or {}
    w = np.zeros(len(locations), dtype=np.float64)
    for i, loc in enumerate(locations):
        if i in cached:
            continue
        try:
            size = os.path.getsize(loc)
            w[i] = gzip_bases_estimate(loc, size) if loc.endswith(".gz") and size >= 18 else size
        except OSError:
            w[i] = 0                     # unreadable: the sketch stage reports it
    return w


def cached_sketches(data_folder: str, names: Sequence[str], s: int, group_size: int = 1000) -> Dict[int, object]:
    """Existing sketches of the drop-in's work directory layout
    (MASH_files/sketches/chunk_<i>/<genome>.msh, groupSize genomes per chunk;
    d_cluster.py:531-542) that match (k, s, seed)."""
    from .d_cluster import _load_cached
    out: Dict[int, object] = {}
    folder = os.path.join(data_folder, "MASH_files", "sketches")
    for idx, name in enumerate(names):
        f = os.path.join(folder, "chunk_%d" % (idx // group_size), name + ".msh")
        if os.path.isfile(f):
            ref = _load_cached(f, s)
            if ref is not None:
                out[idx] = ref
    return out


def sharded_screen_enabled() -> bool:
    """DREPHIP_SCREEN_SHARD=0 turns the sharded screen off: every rank then
    groups all N x s entries itself (the round-5 form)."""
    return os.environ.get("DREPHIP_SCREEN_SHARD", "1") != "0"


def sharded_screen_applies(ctx, N: int) -> bool:
    """Whether this rank's all-pairs call over N genomes takes the sharded
    screen: several ranks, DREPHIP_SCREEN_SHARD not 0, and a screen this
    context would run for N (mode, N >= 4096 in auto, N x s < 2^32).  The
    same on every rank (same N, mode and environment), as it must be: the
    exchange is collective."""
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    return world > 1 and sharded_screen_enabled() and ctx.screen_worth(N, 0)[0]


def allpairs_rows_sharded(ctx, H, NH, N: int, r0: int, r1: int, d_seg: Optional[int], d_denom: Optional[int],
                          stream: int, device) -> float:
    """Rows [r0, r1) with the screen sharded by hash range (every rank calls it:
    collective).  Rank p groups hash part p of W (drephip_screen_part); the
    parts' marked cell words and runs-of-two records go to the ranks owning
    their rows (parallel.exchange_screen_parts, one all-to-all); each rank then
    screens its rows from what it received (drephip_allpairs_device_marked).  The
    pair checks summed over the parts decide the screen as the one-GPU call
    decides it; a dense set takes the dense plan.  d_seg None: a rank without
    rows, which still groups its part and takes part in the exchange.
    Returns the part's screen time (ms; 0 unless the context times kernel 4):
    the marked call's own timings replace it in the context."""
    import torch
    import torch.distributed as dist
    from .parallel import exchange_screen_parts
    world = dist.get_world_size()
    checks, ncells, nrec = ctx.screen_part(H.data_ptr(), NH.data_ptr(), N, dist.get_rank(), world, stream)
    part_ms = ctx.kernel_ms(4)[0]
    cells = torch.empty((max(ncells, 1), 4), dtype=torch.int32, device=device)
    rec = torch.empty((max(nrec, 1), 4), dtype=torch.int32, device=device)
    ctx.screen_part_copy(cells.data_ptr(), rec.data_ptr(), stream)
    starts = [a for a, _ in row_partition(N, world)]                 # every rank's rows (plan())
    cells, recs, total = exchange_screen_parts(cells, ncells, rec, nrec, checks, starts, ctx.screen_geometry())
    if d_seg is None:
        return part_ms
    if ctx.screen_worth(N, total)[1]:
        ctx.allpairs_device_marked(H.data_ptr(), NH.data_ptr(), N, r0, r1, d_seg, d_denom,
                                   cells.data_ptr() if len(cells) else None, len(cells),
                                   recs.data_ptr() if len(recs) else None, len(recs), stream)
    else:                                     # a dense set: the dense plan, as the one-GPU call
        mode = ctx.allpairs_screen
        ctx.set_allpairs_screen(ctx.SCREEN_OFF)
        try:
            ctx.allpairs_device(H.data_ptr(), NH.data_ptr(), N, r0, r1, d_seg, d_denom, stream)
        finally:
            ctx.set_allpairs_screen(mode)
    return part_ms


def hip_allpairs(ctx, stream: int, device):
    """Stage 3: drephip_allpairs_device over this rank's rows, on its GPU --
    with the screen sharded by hash range when it applies
    (allpairs_rows_sharded) instead of every rank sorting all N x s entries."""
    import torch

    def fn(H, NH, p: ShardPlan, out=None):
        # `out`: where the segment goes (a slice of the root's full vector)
        seg = out if out is not None and p.seg_len else torch.zeros(max(p.seg_len, 1), dtype=torch.int16, device=device)
        partial = bool((NH < ctx.s).any().item())
        segd = torch.zeros(max(p.seg_len, 1), dtype=torch.int16, device=device) if partial else None
        dptr = segd.data_ptr() if segd is not None else None
        if sharded_screen_applies(ctx, p.N):
            allpairs_rows_sharded(ctx, H, NH, p.N, p.r0, p.r1, seg.data_ptr() if p.seg_len else None, dptr, stream,
                                  device)
        elif p.seg_len:
            ctx.allpairs_device(H.data_ptr(), NH.data_ptr(), p.N, p.r0, p.r1, seg.data_ptr(), dptr, stream)
        return seg, segd
    return fn


def hip_linkage(ctx, names: Sequence[str], stream: int):
    """Stage 5: drephip_linkage_counts_device on the root GPU, rows in
    sorted-name order (the pivot's order, d_cluster.py:620)."""
    from .d_cluster import linkage_order, linkage_tables

    def fn(common, denom, N, method):
        import torch
        if denom is None:
            dens = np.array([ctx.s])
        else:
            # denominators that occur, by a presence mask over 0..s filled in
            # chunks (a torch.unique of the whole vector would sort 5x10^9
            # entries and hold several GB of extra HBM at 10^5 genomes)
            seen = torch.zeros(ctx.s + 1, dtype=torch.bool, device=denom.device)
            step = 1 << 27
            for a in range(0, denom.numel(), step):
                seen[denom[a:a + step].to(torch.int64) & 0xFFFF] = True
            dens = np.nonzero(seen.cpu().numpy())[0]
        lut, lut_off = linkage_tables(dens, ctx.s)
        return ctx.linkage_counts_device(common.data_ptr(), None if denom is None else denom.data_ptr(), N,
                                         linkage_order(names), lut, lut_off, method, stream)
    return fn


def start_linkage_reserve(link_ctx, N: int, s: int, device, record: Dict):
    """Reserve the root's n x n f64 linkage matrix on a helper thread (80 GB at
    10^5 genomes: ~2 s of hipMalloc once the process has cached memory, 0.5 ms
    at its start), beside the sketch and all-pairs stages.  Skipped when it
    would not leave the stages their HBM: the full sketch matrix, the condensed
    counts (2 B per pair, twice with partial sketches) and a 4 GiB margin.  An
    exception in the thread is recorded in `record['reserve_error']` (the job's
    JSON line), not lost; the linkage then allocates the matrix itself.
    Returns the started thread, or None when skipped."""
    import threading
    import torch
    need = N * N * 8
    stages = N * s * 8 + 4 * (N * (N - 1) // 2) + (4 << 30)
    free, _ = torch.cuda.mem_get_info(device)
    if need + stages > free:
        record["reserve_skipped"] = ("matrix %.1f GB + stages %.1f GB > free HBM %.1f GB"
                                     % (need / 1e9, stages / 1e9, free / 1e9))
        return None

    def run():
        t0 = time.perf_counter()
        try:
            link_ctx.linkage_reserve(N)
            record["reserve_s"] = time.perf_counter() - t0
        except Exception as e:          # recorded; the linkage allocates on its own
            record["reserve_error"] = "%s: %s" % (type(e).__name__, e)
    t = threading.Thread(target=run, daemon=True)
    t.start()
    return t


def synthetic_names(N: int) -> List[str]:
    """Genome names of the synthetic workload: sorting them keeps index order."""
    return ["synthetic_%07d.fna" % i for i in range(N)]


def main(argv: Optional[Sequence[str]] = None) -> int:
    """configs[3] as one job: `python -m torch.distributed.run --nproc-per-node 8
    --master-addr 127.0.0.1 -m drep_amd.distributed --genomes 100000`
    (synthetic genomes), or over real FASTA files with --bdb Bdb.csv / --files
    list.txt (and --data-folder for dRep's cached .msh sketches).  Prints one
    JSON line (rank 0); --out stores the condensed counts, the primary_linkage
    pickle and the primary Cdb in drep_amd.store formats."""
    import argparse
    import torch
    import torch.distributed as dist
    from . import _lib
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=100_000)
    ap.add_argument("--genome-bp", type=int, default=5_000_000)
    ap.add_argument("--sketch", type=int, default=1000)
    ap.add_argument("--family-size", type=int, default=100)
    ap.add_argument("--seed", type=int, default=0xD2E9)
    ap.add_argument("--method", default="average")
    ap.add_argument("--P-ani", type=float, default=0.9)
    ap.add_argument("--out", default=None, help="work-directory data folder to store the results in")
    ap.add_argument("--bdb", default=None, help="genomes from a dRep Bdb table (CSV: genome, location)")
    ap.add_argument("--files", default=None, help="genomes from a text file of FASTA paths, one per line")
    ap.add_argument("--data-folder", default=None,
                    help="reuse cached sketches under <data-folder>/MASH_files/sketches/chunk_<i>/ (dRep layout)")
    ap.add_argument("--group-size", type=int, default=1000, help="genomes per sketch chunk folder (dRep groupSize)")
    ap.add_argument("--processors", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0),
                    help="host threads for FASTA ingest per rank (0 = all)")
    a = ap.parse_args(argv)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = os.environ.get("DREPHIP_DIST_BACKEND", "nccl")      # nccl = RCCL over xGMI
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    ctx = _lib.Context(device=local, k=21, s=a.sketch, seed=42)
    stream = torch.cuda.current_stream(dev).cuda_stream
    from_files = bool(a.bdb or a.files)
    if from_files:
        names, locations = read_genome_list(a.bdb, a.files)
        N = len(names)
        lengths = np.zeros(N, dtype=np.uint64)
        cached = cached_sketches(a.data_folder, names, a.sketch, a.group_size) if a.data_folder else {}
        sketch_fn = hip_file_sketcher(ctx, locations, a.processors, dev, cached, lengths)
        # the root's weights for every rank: a rank that saw another file size
        # or another cached set would build another shard plan, and the
        # gathered rows would land in the wrong genome order without an error
        box = [file_weights(locations, cached) if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(box, src=0)
        weights = box[0]
    else:
        N = a.genomes
        names = locations = synthetic_names(N)
        lengths = np.full(N, a.genome_bp, np.uint64)
        sketch_fn = hip_synth_sketcher(ctx, a.genome_bp, a.family_size, a.seed, stream, dev)
        weights = None                                   # one length: contiguous equal shards
    # the root's n x n linkage matrix (80 GB at 10^5: ~2 s of hipMalloc) is
    # allocated by a separate context on a helper thread while the sketch and
    # all-pairs stages run, so the serial clustering tail does not pay for it
    link_ctx, reserve = ctx, None
    res_wait: Dict = {}
    if rank == 0 and N >= 2:
        link_ctx = _lib.Context(device=local, k=21, s=a.sketch, seed=42)
        reserve = start_linkage_reserve(link_ctx, N, a.sketch, dev, res_wait)
    linkage_fn = hip_linkage(link_ctx, names, stream)
    if reserve is not None:
        inner = linkage_fn

        def linkage_fn(*args):
            t0 = time.perf_counter()
            reserve.join()
            res_wait["reserve_wait_s"] = time.perf_counter() - t0
            return inner(*args)
    res = run_sharded(N, names, a.sketch, sketch_fn, hip_allpairs(ctx, stream, dev), linkage_fn,
                      a.method, a.P_ani, sync=lambda: torch.cuda.synchronize(dev), weights=weights)
    if from_files and world > 1:
        # every rank filled its shard's lengths: the root takes the element-wise max
        allv = [None] * world
        dist.all_gather_object(allv, lengths)
        lengths = np.maximum.reduce(allv)
    if rank == 0:
        out = {"job": "configs[3]-style sharded Mash step + primary clustering", "genomes": N,
               "input": ("files (%d cached sketches)" % len(cached)) if from_files else "synthetic",
               "genome_bp": None if from_files else a.genome_bp, "sketch": a.sketch, "n_gpus": world,
               "backend": backend, "method": a.method, "P_ani": a.P_ani, "times": res["times"],
               "pairs": N * (N - 1) // 2, "primary_clusters": int(res["Cdb"]["primary_cluster"].nunique())}
        out.update(res_wait)
        if weights is not None:          # the sketch shards' work (file bytes) per rank
            out["shard_weights"] = [float(weights[m].sum()) for m in balanced_shards(weights, world)]
            out["shard_genomes"] = [int(len(m)) for m in balanced_shards(weights, world)]
        out["linkage_phases_s"] = link_ctx.linkage_stats()
        t = res["times"]
        out["pairs_per_s_job"] = out["pairs"] / sum(v for k, v in t.items())
        if a.out:
            from .d_cluster import CondensedMash
            from .store import store_condensed, store_primary_linkage
            os.makedirs(a.out, exist_ok=True)
            cm = CondensedMash(list(names), list(locations), res["common"].cpu().numpy().view(np.uint16),
                               None if res["denom"] is None else res["denom"].cpu().numpy().view(np.uint16),
                               res["nhash"].cpu().numpy().view(np.uint32), lengths, a.sketch)
            store_condensed(a.out, cm)
            store_primary_linkage(a.out, res["linkage"], None, res["arguments"])
            res["Cdb"].to_csv(os.path.join(a.out, "primary_Cdb.csv"), index=False)
            out["stored"] = a.out
        print(json.dumps(out), flush=True)
    if link_ctx is not ctx:
        link_ctx.close()
    ctx.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
