"""Multi-GPU sharding of the Mash step: one process per GPU (torchrun).

The reference runs everything in one process (mash dist -p threads,
d_cluster.py:570); it has no distributed code.  On a node of MI355X the step
splits as:

* sketch: genome shards -- contiguous and of equal count for synthetic
  genomes of one length, balanced by file size (balanced_shards) for FASTA
  inputs -- each rank sketches its own genomes;
* exchange: ONE collective, an all-gather of the uint64[N/W][s] sketch shards
  and their nhash counts (RCCL over xGMI with the "nccl" backend; gloo on CPU
  in the tests);
* all-pairs: contiguous row ranges of the upper triangle balanced by pair
  count; each rank writes one contiguous segment of the condensed output, so
  the result needs no collective (segments are concatenated on the host).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def genome_shard(N: int, world: int, rank: int) -> Tuple[int, int, int]:
    """(g0, g1, nmax): rank's contiguous genome range and the padded shard size
    every rank uses so the all-gather chunks are equal."""
    nmax = (N + world - 1) // world
    g0 = min(N, rank * nmax)
    g1 = min(N, g0 + nmax)
    return g0, g1, nmax


def balanced_shards(weights: Sequence[float], world: int) -> List[np.ndarray]:
    """Genome shards balanced by work ("greedily by total
    bases"): genomes in decreasing weight order, each to the rank with the
    least total so far (ties: the lowest rank), i.e. LPT list scheduling.
    Every rank's total is then within one genome's weight of every other's
    (the rank that ends heaviest was the lightest when it took its last
    genome).  Genomes of zero weight (cached sketches, unreadable files) cost
    no sketch work but still a row of the all-gather, which pads every shard
    to the largest: they go, after the others, each to the rank holding the
    fewest genomes (ties in weight likewise go to the rank holding fewer), so
    an all-cached rerun gets equal counts instead of every genome on rank 0.
    Returns each rank's genome indices, ascending.  The reference fans the
    genomes out over a thread pool in Bdb order (drep/d_cluster.py:527-549),
    where no balance is needed."""
    import heapq
    w = np.asarray(weights, dtype=np.float64)
    order = np.argsort(-w, kind="stable")
    heap = [(0.0, 0, r) for r in range(world)]
    heapq.heapify(heap)
    members: List[List[int]] = [[] for _ in range(world)]
    zeros = []
    for g in order:
        if not w[g] > 0:
            zeros.append(int(g))
            continue
        tot, cnt, r = heapq.heappop(heap)
        members[r].append(int(g))
        heapq.heappush(heap, (tot + float(w[g]), cnt + 1, r))
    by_count = [(len(members[r]), r) for r in range(world)]
    heapq.heapify(by_count)
    for g in zeros:
        cnt, r = heapq.heappop(by_count)
        members[r].append(g)
        heapq.heappush(by_count, (cnt + 1, r))
    return [np.sort(np.asarray(m, dtype=np.int64)) for m in members]


def shard_layout(shards: Sequence[np.ndarray], N: int) -> Tuple[int, np.ndarray]:
    """(nmax, pos) for an all-gather of shards padded to nmax rows: genome g
    lands at gathered row pos[g] = rank * nmax + (its slot in the shard)."""
    nmax = max(1, max(len(m) for m in shards))
    pos = np.full(N, -1, dtype=np.int64)
    for r, m in enumerate(shards):
        pos[m] = r * nmax + np.arange(len(m))
    if (pos < 0).any():
        raise ValueError("the shards do not cover every genome")
    return nmax, pos


def cond_start(i: int, N: int) -> int:
    """Condensed index of pair (i, i+1) (scipy squareform order)."""
    return i * N - i * (i + 1) // 2


def row_partition(N: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous row ranges [r0, r1) of the upper triangle with near-equal
    pair counts (row i has N-1-i pairs)."""
    pairs = np.arange(N - 1, -1, -1, dtype=np.float64)
    cum = np.concatenate([[0.0], np.cumsum(pairs)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        t = total * r / world
        i = int(np.searchsorted(cum, t))
        if i > 0 and abs(cum[i - 1] - t) <= abs(cum[min(i, N)] - t):
            i -= 1                                   # nearest row boundary
        bounds.append(i)
    bounds.append(N)
    for r in range(1, len(bounds)):
        bounds[r] = max(bounds[r], bounds[r - 1])
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def segment_size(N: int, r0: int, r1: int) -> int:
    """Number of condensed pairs in rows [r0, r1)."""
    if N < 2 or r0 >= min(r1, N - 1):
        return 0
    return cond_start(min(r1, N - 1), N) - cond_start(r0, N)


def gather_sketches(local_h, local_n, group=None):
    """All-gather equal-size sketch shards (torch tensors on the process's
    device: int64 [nmax, s] viewed as uint64, int32 [nmax]).  Returns the
    gathered [world*nmax, s] and [world*nmax] tensors; rows >= N are padding.
    One all-gather (RCCL over xGMI with the nccl backend) of [nmax, s+1]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    nmax, s = local_h.shape
    # one collective: the count rides along as an extra int64 column
    packed = torch.empty((nmax, s + 1), dtype=torch.int64, device=local_h.device)
    packed[:, :s] = local_h
    packed[:, s] = local_n.to(torch.int64)
    gathered = torch.empty((world * nmax, s + 1), dtype=torch.int64, device=local_h.device)
    dist.all_gather_into_tensor(gathered, packed, group=group)
    all_h = gathered[:, :s].contiguous()
    all_n = gathered[:, s].to(local_n.dtype).contiguous()
    return all_h, all_n


def exchange_screen_parts(bitmap, records, nrec: int, checks: int, row_starts=None, group=None):
    """The sharded screen's exchange (include/drephip.h drephip_screen_part).

    bitmap: this rank's part bitmap (uint32 words as int32, equal size on every
    rank); records: its runs-of-two records ([>= nrec, 4] int32, {a, b, pos,
    0}); checks: its pair checks.  Returns (bitmaps [world, words] in part
    order, the records this rank needs [n, 4], total pair checks).

    The bitmaps are all-gathered (every rank needs every part's cells of its
    rows; one part's bitmap is ceil(N/R) x ceil(N/32) words).  The records go
    to their owners only: with row_starts (every rank's first row, ascending)
    record {a, ...} goes to the rank whose rows hold a, by one all-to-all;
    without, every rank gets every record (an all-gather).  RCCL over xGMI with
    nccl; gloo in rehearsals (records staged through the host there)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = bitmap.device
    rec = records[:nrec]
    if row_starts is not None:
        starts = torch.as_tensor(np.asarray(row_starts, np.int64), device=dev)
        owner = torch.searchsorted(starts, rec[:, 0].to(torch.int64), right=True) - 1
        order = torch.argsort(owner, stable=True)
        rec = rec[order]
        send = torch.bincount(owner, minlength=world).to(torch.int64)
    else:
        send = torch.full((world,), nrec, dtype=torch.int64, device=dev)
    # (outputs shaped [world * input rows, ...]: gloo splits them along dim 0)
    meta = torch.cat([send, torch.tensor([nrec, checks], dtype=torch.int64, device=dev)])
    allm = torch.empty(world * (world + 2), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allm, meta, group=group)
    allm = allm.view(world, world + 2).cpu()
    total_checks = int(allm[:, world + 1].sum())
    bms = torch.empty(world * bitmap.numel(), dtype=bitmap.dtype, device=dev)
    dist.all_gather_into_tensor(bms, bitmap.reshape(-1), group=group)
    bms = bms.view(world, bitmap.numel())
    if row_starts is not None:
        send_sizes = [int(x) for x in allm[rank, :world]]
        recv_sizes = [int(x) for x in allm[:, rank]]
        host = dist.get_backend(group) == "gloo" and rec.is_cuda
        src = rec.contiguous().cpu() if host else rec.contiguous()
        out = torch.empty((sum(recv_sizes), 4), dtype=torch.int32, device=src.device)
        dist.all_to_all_single(out, src, output_split_sizes=recv_sizes, input_split_sizes=send_sizes, group=group)
        return bms, out.to(dev).contiguous(), total_checks
    counts = [int(c) for c in allm[:, world]]
    cmax = max(max(counts), 1)
    padded = torch.zeros((cmax, 4), dtype=torch.int32, device=dev)
    if nrec:
        padded[:nrec] = rec
    recs = torch.empty((world * cmax, 4), dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(recs, padded, group=group)
    recs = recs.view(world, cmax, 4)
    keep = torch.cat([recs[p, :counts[p]] for p in range(world)]) if sum(counts) else recs[0, :0]
    return bms, keep.contiguous(), total_checks


def assemble_condensed(N: int, segments: Sequence[np.ndarray], world: int) -> np.ndarray:
    """Concatenate per-rank condensed segments (rank order) into the full
    condensed vector, checking every segment has its expected size."""
    parts = row_partition(N, world)
    out = []
    for (r0, r1), seg in zip(parts, segments):
        want = segment_size(N, r0, r1)
        if len(seg) != want:
            raise ValueError("segment for rows [%d,%d) has %d pairs, expected %d" % (r0, r1, len(seg), want))
        out.append(np.asarray(seg))
    full = np.concatenate(out) if out else np.zeros(0, np.uint16)
    if len(full) != N * (N - 1) // 2:
        raise ValueError("segments do not cover the triangle")
    return full
