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


ROW_ALIGN = 8      # rank boundaries on multiples of 8 rows: the all-pairs row tiles (1, 2, 4 or 8 rows)


def row_partition(N: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous row ranges [r0, r1) of the upper triangle with near-equal
    pair counts (row i has N-1-i pairs).  Interior boundaries fall on
    multiples of ROW_ALIGN rows (the nearest one), so every rank's row tiles
    are the sharded screen's tiles counted from row 0 (drephip_screen_part):
    its marks map onto a rank's tiles exactly (a boundary inside a tile would
    give the rank the union of two tiles' cells)."""
    pairs = np.arange(N - 1, -1, -1, dtype=np.float64)
    cum = np.concatenate([[0.0], np.cumsum(pairs)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        t = total * r / world
        i = int(np.searchsorted(cum, t))
        if i > 0 and abs(cum[i - 1] - t) <= abs(cum[min(i, N)] - t):
            i -= 1                                   # nearest row boundary
        lo = i - i % ROW_ALIGN
        hi = min(lo + ROW_ALIGN, N)
        i = lo if abs(cum[lo] - t) <= abs(cum[hi] - t) else hi
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


def exchange_screen_parts(cells, ncells: int, records, nrec: int, checks: int, row_starts: Sequence[int],
                          rows_per_tile: int, group=None):
    """The sharded screen's exchange (include/drephip.h drephip_screen_part).

    This rank's part: `ncells` cell words {T, w, bits, 0} (row tile T = rows
    [T R, (T + 1) R)) and `nrec` runs-of-two records {a, b, pos, 0}, as [n, 4]
    int32 tensors (rows past n ignored), and its pair checks.  Each cell goes
    to the rank whose rows hold row T R, each record to the rank whose rows
    hold row a (row_starts: every rank's first row, ascending), by one
    all-to-all; the counts ride an all-gather first (with the checks, whose sum
    decides the screen).  Returns (the cells and the records this rank
    received, in source-part order; the total pair checks).  RCCL over xGMI
    with nccl; gloo in rehearsals (staged through the host there)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = cells.device
    starts = torch.as_tensor(np.asarray(row_starts, np.int64), device=dev)

    def by_owner(t, n, row_of):
        t = t[:n]
        owner = torch.searchsorted(starts, row_of(t), right=True) - 1
        order = torch.argsort(owner, stable=True)
        return t[order], torch.bincount(owner, minlength=world).to(torch.int64)
    c, csend = by_owner(cells, ncells, lambda t: t[:, 0].to(torch.int64) * rows_per_tile)
    r, rsend = by_owner(records, nrec, lambda t: t[:, 0].to(torch.int64))
    # (outputs shaped [world * input rows, ...]: gloo splits them along dim 0)
    meta = torch.cat([csend, rsend, torch.tensor([checks], dtype=torch.int64, device=dev)])
    allm = torch.empty(world * (2 * world + 1), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allm, meta, group=group)
    allm = allm.view(world, 2 * world + 1).cpu()
    total_checks = int(allm[:, 2 * world].sum())
    # one buffer: for each destination its cells, then its records
    cs, rs = [int(x) for x in allm[rank, :world]], [int(x) for x in allm[rank, world:2 * world]]
    co, ro = np.concatenate([[0], np.cumsum(cs)]), np.concatenate([[0], np.cumsum(rs)])
    send = torch.cat([torch.cat([c[co[d]:co[d + 1]], r[ro[d]:ro[d + 1]]]) for d in range(world)]) if world else c
    cin, rin = [int(x) for x in allm[:, rank]], [int(x) for x in allm[:, world + rank]]
    host = dist.get_backend(group) == "gloo" and send.is_cuda
    src = send.contiguous().cpu() if host else send.contiguous()
    out = torch.empty((sum(cin) + sum(rin), 4), dtype=torch.int32, device=src.device)
    dist.all_to_all_single(out, src, output_split_sizes=[a + b for a, b in zip(cin, rin)],
                           input_split_sizes=[a + b for a, b in zip(cs, rs)], group=group)
    out = out.to(dev)
    got_c, got_r, o = [], [], 0
    for p in range(world):
        got_c.append(out[o:o + cin[p]])
        got_r.append(out[o + cin[p]:o + cin[p] + rin[p]])
        o += cin[p] + rin[p]
    return torch.cat(got_c).contiguous(), torch.cat(got_r).contiguous(), total_checks


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
