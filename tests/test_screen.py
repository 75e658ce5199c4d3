"""The shared-hash screen in front of the all-pairs kernels (screen.hip):
every pair that shares no hash is written as Mash's merge gives it (common 0,
denominator min(s, |A| + |B|)), the others by the LIST kernels.  Checked bit
for bit against the C oracle's Mash merge (reference: `mash dist`,
drep/d_cluster.py:569-573) and against the unscreened (dense) path, on
sketches built to stress it: families sharing values at every rank position,
partial sketches, hashes that agree in their low 32 bits only (the sort key),
values shared by many genomes, genomes sharing nothing, and row segments
(the sharded path's slices)."""
import numpy as np
import pytest

import oracle
from drep_amd import _lib

pytestmark = pytest.mark.gpu
UMAX = np.iinfo(np.uint64).max


def planted_sketches(N, s, seed, fam=6, partial_every=7, lo_twins=40, hub=True):
    """N sorted sketches: families of `fam` genomes draw from a shared pool
    (so family members share hashes anywhere in the rank order), every
    partial_every-th genome is partial, `lo_twins` hashes are copied to
    another genome with only their high word changed (equal sort keys, no
    shared hash), and one hub value sits in a third of all genomes."""
    rng = np.random.default_rng(seed)
    H = np.full((N, s), UMAX, dtype=np.uint64)
    NH = np.zeros(N, dtype=np.uint32)
    hubv = np.uint64(rng.integers(1, UMAX, dtype=np.uint64))
    pools = {}
    for g in range(N):
        f = g // fam
        if f not in pools:
            pools[f] = rng.integers(1, UMAX, size=3 * s, dtype=np.uint64)     # the whole 64-bit range
        own = rng.integers(1, UMAX, size=s, dtype=np.uint64)
        take = rng.random(3 * s) < 0.3
        vals = np.unique(np.concatenate([pools[f][take], own] + ([np.array([hubv])] if hub and g % 3 == 0 else [])))
        n = s if g % partial_every else int(rng.integers(1, s))
        vals = vals[:n]
        H[g, :len(vals)] = vals
        NH[g] = len(vals)
    for _ in range(lo_twins):
        a, b = rng.integers(0, N, 2)
        if a == b or NH[a] == 0 or NH[b] == 0:
            continue
        v = H[a, rng.integers(0, NH[a])]
        twin = (v & np.uint64(0xFFFFFFFF)) | (np.uint64(rng.integers(1, 1 << 32)) << np.uint64(32))
        if twin in H[b, :NH[b]] or twin in H[a, :NH[a]]:
            continue
        row = np.sort(np.concatenate([H[b, :NH[b]], [twin]]))[:s]
        H[b, :] = UMAX
        H[b, :len(row)] = row
        NH[b] = len(row)
    return H, NH


def run(ctx, H, NH, mode, want_denom=True):
    ctx.set_allpairs_screen(mode)
    c, d = ctx.allpairs(H, NH, want_denom=want_denom)
    return c, d, ctx.screen_stats()


@pytest.mark.parametrize("s,N", [(64, 300), (1000, 200), (2048, 96), (4096, 80)])
def test_screen_matches_oracle_and_dense(s, N):
    H, NH = planted_sketches(N, s, seed=s + N)
    oc, od = oracle.allpairs(H, NH, s, threads=8)
    with _lib.Context(0, 21, s, 42) as ctx:
        c, d, st = run(ctx, H, NH, ctx.SCREEN_ON)
        assert st["used"] and st["marked"] > 0 and st["entries"] == int(NH.sum())
        assert np.array_equal(c, oc) and np.array_equal(d, od)
        c2, d2, st2 = run(ctx, H, NH, ctx.SCREEN_OFF)
        assert not st2["used"]
        assert np.array_equal(c2, c) and np.array_equal(d2, d)
    assert (oc > 0).sum() > N          # families and the hub: many pairs share hashes
    assert (oc == 0).sum() > N         # and many share none


def test_screen_nothing_shared_and_all_shared():
    s, N = 200, 150
    rng = np.random.default_rng(11)
    H = np.sort(rng.permutation(np.arange(1, N * s + 1, dtype=np.uint64) * np.uint64(7919)).reshape(N, s), axis=1)
    NH = np.full(N, s, dtype=np.uint32)
    NH[::5] = 37
    H[::5, 37:] = UMAX
    with _lib.Context(0, 21, s, 42) as ctx:
        c, d, st = run(ctx, H, NH, ctx.SCREEN_ON)
        assert st["used"] and st["marked"] == 0
        oc, od = oracle.allpairs(H, NH, s, threads=8)
        assert np.array_equal(c, oc) and np.array_equal(d, od) and c.max() == 0
        # every genome identical: every cell marked
        same = np.tile(np.sort(rng.integers(1, 1 << 60, size=s, dtype=np.uint64)), (N, 1))
        c, d, st = run(ctx, same, np.full(N, s, np.uint32), ctx.SCREEN_ON)
        assert (c == s).all() and (d == s).all()
        # auto mode refuses the all-shared set (the dense path is cheaper)
        ctx.set_allpairs_screen(ctx.SCREEN_AUTO)
        import os
        os.environ["DREPHIP_SCREEN_MIN_N"] = "2"
        try:
            c, d = ctx.allpairs(same, np.full(N, s, np.uint32), want_denom=True)
            assert not ctx.screen_stats()["used"] and (c == s).all()
        finally:
            os.environ.pop("DREPHIP_SCREEN_MIN_N")


@pytest.mark.parametrize("s", [1000, 4096])
def test_screen_row_segments(s):
    """Row ranges (a rank's slice of the triangle): the screen marks only
    pairs whose smaller genome is a row of the call."""
    N = 120
    H, NH = planted_sketches(N, s, seed=5 * s)
    oc, od = oracle.allpairs(H, NH, s, threads=8)

    def start(i):
        return i * N - i * (i + 1) // 2
    with _lib.Context(0, 21, s, 42) as ctx:
        ctx.set_allpairs_screen(ctx.SCREEN_ON)
        for r0, r1 in ((0, 17), (17, 64), (64, 119), (118, 119)):
            n = start(r1) - start(r0)
            co = np.zeros(n, np.uint16)
            do = np.zeros(n, np.uint16)
            ctx.allpairs_rows(H, NH, r0, r1, co, do)
            assert ctx.screen_stats()["used"]
            assert np.array_equal(co, oc[start(r0):start(r1)]), (r0, r1)
            assert np.array_equal(do, od[start(r0):start(r1)]), (r0, r1)


def test_screen_auto_on_family_sets():
    """Auto mode on sketches of synthetic genome families (the bench's
    generator; many unrelated pairs): the screen is taken and gives the
    oracle's counts."""
    import os
    h, nh = oracle.sketch_synth(0, 200, 300_000, seed=9, family_size=20, s=1000, threads=8)
    os.environ["DREPHIP_SCREEN_MIN_N"] = "2"
    try:
        with _lib.Context(0, 21, 1000, 42) as ctx:
            c, d = ctx.allpairs(h, nh, want_denom=True)
            st = ctx.screen_stats()
    finally:
        os.environ.pop("DREPHIP_SCREEN_MIN_N")
    oc, od = oracle.allpairs(h, nh, 1000, threads=8)
    assert np.array_equal(c, oc) and np.array_equal(d, od)
    assert st["used"] and st["entries"] == int(nh.sum())


def test_screen_single_shared_hash_pairs():
    """Pairs of otherwise unrelated genomes that share exactly one hash are
    written by the screen itself (count = 1 iff the hash's rank in A u B,
    i + j, is below s); pairs sharing two such hashes, or with a partial
    sketch, go to the kernel.  Planted at positions on both sides of
    i + j = s, checked against the oracle."""
    s, N = 256, 400
    rng = np.random.default_rng(21)
    H = np.sort(rng.integers(1, 1 << 62, size=(N, s), dtype=np.uint64), axis=1)     # random: no value shared by chance
    NH = np.full(N, s, dtype=np.uint32)
    for g in range(0, N, 9):                       # partial sketches
        NH[g] = rng.integers(s // 3, s)
        H[g, NH[g]:] = UMAX
    planted = 0
    for _ in range(600):
        a, b = sorted(rng.choice(N, 2, replace=False))
        for _k in range(1 if rng.random() < 0.8 else 2):           # one shared hash, sometimes two
            i, j = int(rng.integers(0, NH[a])), int(rng.integers(0, NH[b]))
            v = H[a, i]
            if v in H[b, :NH[b]]:
                continue
            row = np.sort(np.concatenate([np.delete(H[b, :NH[b]], j), [v]]))
            H[b, :NH[b]] = row
            planted += 1
    oc, od = oracle.allpairs(H, NH, s, threads=8)
    with _lib.Context(0, 21, s, 42) as ctx:
        c, d, st = run(ctx, H, NH, ctx.SCREEN_ON)
        assert st["used"] and st["simple"] > 100, st
        assert np.array_equal(c, oc) and np.array_equal(d, od)
        c2, d2, _ = run(ctx, H, NH, ctx.SCREEN_OFF)
        assert np.array_equal(c2, oc) and np.array_equal(d2, od)
    assert planted > 500 and (oc == 1).sum() > 100 and ((oc == 0) & (od == s)).sum() > 1000


@pytest.mark.parametrize("s,N", [(300, 400), (4096, 264)])
def test_screen_light_cells(s, N, monkeypatch):
    """Light cells (k_screen_light), planted as configs[4] has them: families
    of 8 genomes share 30 values each (heavy cells); a value shared by chance
    between members of two families (a run of >= 3 entries) gives their
    cross pairs exactly one shared hash (light cells), at ranks on both sides
    of i + j = s; hub values in ~70 genomes across families (runs longer than
    a wave: row tiles straddle x blocks); some family pairs linked by two chance
    values, or by a chance value and a two-genome value (heavy); partial
    sketches (heavy); values that agree in their low word only.  The screen
    writes the light pairs itself: bit-exact against the oracle and against
    the screen without the light path, which leaves more cells to the kernel."""
    rng = np.random.default_rng(s + N)
    F = 8
    H = np.sort(rng.integers(1, 1 << 62, size=(N, s), dtype=np.uint64), axis=1)
    NH = np.full(N, s, dtype=np.uint32)
    for g in range(5, N, 29):
        NH[g] = rng.integers(s // 3, s)
        H[g, NH[g]:] = UMAX

    def plant(members, v):
        for g in members:
            if v in H[g, :NH[g]]:
                continue
            j = int(rng.integers(0, NH[g]))
            row = np.sort(np.concatenate([np.delete(H[g, :NH[g]], j), [v]]))
            H[g, :NH[g]] = row

    def fam(f):
        return np.arange(f * F, min(N, f * F + F))
    nf = N // F
    for f in range(nf):
        for _ in range(30):
            plant(fam(f), np.uint64(rng.integers(1, 1 << 62)))
    pairs = rng.permutation([(a, b) for a in range(nf) for b in range(a + 1, nf)])
    for a, b in pairs[:60]:                              # one chance value: light cross pairs
        ma = rng.choice(fam(a), int(rng.integers(1, F + 1)), replace=False)
        mb = rng.choice(fam(b), int(rng.integers(2, F + 1)), replace=False)
        plant(np.concatenate([ma, mb]), np.uint64(rng.integers(1, 1 << 62)))
    for a, b in pairs[60:70]:                            # two chance values: heavy
        for _ in range(2):
            plant(np.concatenate([fam(a)[:3], fam(b)[:3]]), np.uint64(rng.integers(1, 1 << 62)))
    for a, b in pairs[:8]:                               # a two-genome value on top of a chance one
        plant([fam(a)[0], fam(b)[-1]], np.uint64(rng.integers(1, 1 << 62)))
    for _ in range(3):                                   # hubs: runs of ~70
        plant(rng.choice(N, 70, replace=False), np.uint64(rng.integers(1, 1 << 62)))
    for _ in range(30):                                  # low-word twins: equal sort keys, no shared hash
        a, b = rng.choice(N, 2, replace=False)
        v = H[a, rng.integers(0, NH[a])]
        plant([b], (v & np.uint64(0xFFFFFFFF)) | (np.uint64(rng.integers(1, 1 << 30)) << np.uint64(32)))
    oc, od = oracle.allpairs(H, NH, s, threads=8)

    def start(i):
        return i * N - i * (i + 1) // 2
    with _lib.Context(0, 21, s, 42) as ctx:
        monkeypatch.setenv("DREPHIP_SCREEN_LIGHT", "1")        # (by default only with the band kernel, s > 2048)
        c, d, st = run(ctx, H, NH, ctx.SCREEN_ON)
        assert np.array_equal(c, oc) and np.array_equal(d, od)
        # row ranges (a sharded rank's slice: the marking walks only the part of
        # each run -- hubs span several 64-entry blocks -- among its rows)
        for r0, r1 in ((0, N // 3), (N // 3, 2 * N // 3 + 5), (2 * N // 3 + 5, N - 1)):
            n = start(r1) - start(r0)
            co, do = np.zeros(n, np.uint16), np.zeros(n, np.uint16)
            ctx.allpairs_rows(H, NH, r0, r1, co, do)
            assert np.array_equal(co, oc[start(r0):start(r1)]) and np.array_equal(do, od[start(r0):start(r1)]), (r0, r1)
        monkeypatch.setenv("DREPHIP_SCREEN_LIGHT", "0")
        c2, d2, st2 = run(ctx, H, NH, ctx.SCREEN_ON)
        assert np.array_equal(c2, oc) and np.array_equal(d2, od)
        monkeypatch.delenv("DREPHIP_SCREEN_LIGHT")
        _, _, st3 = run(ctx, H, NH, ctx.SCREEN_ON)            # the default: light with the band kernel only
        assert (st3["simple"], st3["marked"]) == ((st["simple"], st["marked"]) if s > 2048 else (st2["simple"], st2["marked"]))
    # the light path wrote pairs itself and left fewer cells to the kernel
    assert st["simple"] > st2["simple"] + 500 and st["marked"] < st2["marked"] - 200, (st, st2)
    assert (oc == 1).sum() > 500 and ((oc == 0) & (od == s)).sum() > 1000


def test_screen_mode_argument_checked():
    with _lib.Context(0, 21, 1000, 42) as ctx:
        with pytest.raises(_lib.DrepHipError, match="unknown screen mode"):
            ctx.set_allpairs_screen(3)
        ctx.set_allpairs_screen(ctx.SCREEN_AUTO)
        h = np.sort(np.random.default_rng(1).integers(1, 1 << 62, size=(3, 1000), dtype=np.uint64), axis=1)
        ctx.allpairs(h, np.full(3, 1000, np.uint32))
        assert not ctx.screen_stats()["used"]            # auto: N < 4096


def sharded_screen(ctx, dH, dNH, N, W, ranges, want_denom=True):
    """The sharded screen on one GPU, as a W-rank job runs it: every part
    grouped (drephip_screen_part) and copied out, the parts' cell words and
    records concatenated (each rank receives its own; the call ignores other
    rows'), each row range screened from them (drephip_allpairs_device_marked).
    Returns the segments, the summed pair checks and the records per part."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    cells, recs, checks, nrecs = [], [], 0, []
    for p in range(W):
        c, nc, n = ctx.screen_part(dH.data_ptr(), dNH.data_ptr(), N, p, W, st)
        cl = torch.empty((max(nc, 1), 4), dtype=torch.int32, device="cuda")
        rec = torch.empty((max(n, 1), 4), dtype=torch.int32, device="cuda")
        ctx.screen_part_copy(cl.data_ptr(), rec.data_ptr(), st)
        cells.append(cl[:nc])
        recs.append(rec[:n])
        checks += c
        nrecs.append(n)
    cells = torch.cat(cells).contiguous()
    recs = torch.cat(recs).contiguous()

    def start(i):
        return i * N - i * (i + 1) // 2
    out = []
    for r0, r1 in ranges:
        n = start(r1) - start(r0)
        co = torch.zeros(max(n, 1), dtype=torch.int16, device="cuda")
        do = torch.zeros(max(n, 1), dtype=torch.int16, device="cuda") if want_denom else None
        ctx.allpairs_device_marked(dH.data_ptr(), dNH.data_ptr(), N, r0, r1, co.data_ptr(),
                                   do.data_ptr() if do is not None else None,
                                   cells.data_ptr() if len(cells) else None, len(cells),
                                   recs.data_ptr() if len(recs) else None, len(recs), st)
        assert ctx.screen_stats()["used"]
        torch.cuda.synchronize()
        out.append((co[:n].cpu().numpy().view(np.uint16), do[:n].cpu().numpy().view(np.uint16) if do is not None else None))
    return out, checks, nrecs


@pytest.mark.parametrize("s,N", [(64, 300), (1000, 200), (4096, 80)])
@pytest.mark.parametrize("W", [1, 2, 3, 8])
def test_sharded_screen_matches_oracle(s, N, W):
    """The sharded screen (one hash part per rank, marks routed to row
    owners): every rank's rows -- the job's row partition (tile-aligned), and
    ranges that start off a row tile boundary (a part's tile then covers two
    of the range's) -- bit-exact against the oracle, on the planted sketches
    (families, partial sketches, low-word twins, a hub in a third of the
    genomes); the parts' pair checks are at most the one-call screen's."""
    import torch
    from drep_amd import parallel
    H, NH = planted_sketches(N, s, seed=s + N + W)
    oc, od = oracle.allpairs(H, NH, s, threads=8)
    dH = torch.from_numpy(H.view(np.int64)).cuda()
    dNH = torch.from_numpy(NH.view(np.int32)).cuda()

    def start(i):
        return i * N - i * (i + 1) // 2
    with _lib.Context(0, 21, s, 42) as ctx:
        ctx.set_allpairs_screen(ctx.SCREEN_ON)
        ranges = [(a, min(b, N - 1)) for a, b in parallel.row_partition(N, W) if a < N - 1]
        ranges += [(1, 6), (7, N // 2 + 3), (N - 9, N - 1)]
        segs, checks, nrecs = sharded_screen(ctx, dH, dNH, N, W, ranges)
        for (r0, r1), (co, do) in zip(ranges, segs):
            assert np.array_equal(co, oc[start(r0):start(r1)]), (r0, r1)
            assert np.array_equal(do, od[start(r0):start(r1)]), (r0, r1)
        ctx.allpairs(H, NH, want_denom=True)
        # a run of keys equal in their low word only may span parts (its
        # hashes' high words differ): the parts check no more pairs than one call
        assert 0 < checks <= ctx.screen_stats()["checks"]
        assert ctx.screen_worth(N, checks) == (True, True)           # mode ON
    assert sum(nrecs) > 0 and (oc > 0).sum() > N


def test_sharded_screen_single_shared_hash_pairs():
    """Pairs sharing exactly one hash (runs of two) whose runs land in
    different parts: a pair held by two runs of two in two parts must reach
    the kernel, one held by a single run is written by the screen -- the
    records of every part meet in the owner's pair map."""
    import torch
    s, N = 256, 400
    rng = np.random.default_rng(33)
    H = np.sort(rng.integers(1, UMAX, size=(N, s), dtype=np.uint64), axis=1)
    NH = np.full(N, s, dtype=np.uint32)
    for g in range(0, N, 11):
        NH[g] = rng.integers(s // 3, s)
        H[g, NH[g]:] = UMAX
    for _ in range(700):
        a, b = sorted(rng.choice(N, 2, replace=False))
        for _k in range(1 if rng.random() < 0.7 else 2):
            i, j = int(rng.integers(0, NH[a])), int(rng.integers(0, NH[b]))
            v = H[a, i]
            if v in H[b, :NH[b]]:
                continue
            H[b, :NH[b]] = np.sort(np.concatenate([np.delete(H[b, :NH[b]], j), [v]]))
    oc, od = oracle.allpairs(H, NH, s, threads=8)
    dH = torch.from_numpy(H.view(np.int64)).cuda()
    dNH = torch.from_numpy(NH.view(np.int32)).cuda()
    with _lib.Context(0, 21, s, 42) as ctx:
        ctx.set_allpairs_screen(ctx.SCREEN_ON)
        for W in (2, 5):
            segs, _, nrecs = sharded_screen(ctx, dH, dNH, N, W, [(0, N - 1)])
            assert np.array_equal(segs[0][0], oc) and np.array_equal(segs[0][1], od), W
            assert min(nrecs) > 50
            assert ctx.screen_stats()["simple"] > 300


@pytest.mark.parametrize("s,N,W", [(16, 1500, 8), (16, 1500, 3), (3, 600, 8)])
def test_sharded_screen_value_cuts(s, N, W):
    """The parts are value ranges cut at medians of per-sketch quantiles
    (k_part_bounds): more genomes than the 1024 sampled ones, empty and
    partial sketches among them, sketches of genomes of different sizes (a
    small genome's bottom-s reaches higher values), and s = 3 with 8 parts
    (equal cuts: empty parts).  Every hash shared anywhere in the value range
    must be grouped by exactly one part: bit-exact against the oracle."""
    import torch
    rng = np.random.default_rng(s * N + W)
    pool = rng.integers(1, UMAX, size=20 * s, dtype=np.uint64)
    H = np.full((N, s), UMAX, dtype=np.uint64)
    NH = np.zeros(N, dtype=np.uint32)
    for g in range(N):
        if g % 7 == 3:
            continue                                          # empty sketch
        scale = np.uint64(1 << int(rng.integers(0, 6)))       # "genome size": values up to UMAX / scale
        own = rng.integers(1, UMAX, size=s, dtype=np.uint64) // scale
        vals = np.unique(np.concatenate([rng.choice(pool, s // 2 + 1) // scale, own]))
        n = s if g % 5 else int(rng.integers(1, s + 1))
        H[g, :min(n, len(vals))] = vals[:n]
        NH[g] = min(n, len(vals))
    oc, od = oracle.allpairs(H, NH, s, threads=8)
    dH = torch.from_numpy(H.view(np.int64)).cuda()
    dNH = torch.from_numpy(NH.view(np.int32)).cuda()
    from drep_amd import parallel

    def start(i):
        return i * N - i * (i + 1) // 2
    with _lib.Context(0, 21, s, 42) as ctx:
        ctx.set_allpairs_screen(ctx.SCREEN_ON)
        ranges = [(a, min(b, N - 1)) for a, b in parallel.row_partition(N, W) if a < N - 1]
        segs, checks, _ = sharded_screen(ctx, dH, dNH, N, W, ranges)
        for (r0, r1), (co, do) in zip(ranges, segs):
            assert np.array_equal(co, oc[start(r0):start(r1)]), (r0, r1)
            assert np.array_equal(do, od[start(r0):start(r1)]), (r0, r1)
        assert checks > 0
    assert (oc > 0).sum() > N // 2


@pytest.mark.parametrize("s,N,edge", [(600, 300, False), (1000, 240, False), (1000, 240, True), (2048, 120, True),
                                      (64, 500, False), (64, 500, True)])
def test_dense_verdict_chunk_masks(s, N, edge):
    """After the screen's dense verdict the whole-row kernel skips the
    high-word check on chunks whose low words no other hash of the set shares
    (k_cmask_*, probe_rows_v<EXACT = false>).  One-species sets (the verdict
    must be dense) with low-word twins -- hashes that share a low word and are
    each held by many genomes, sometimes both by one -- partial sketches, and s
    not a multiple of 64 (chunks past s read zeros), and (edge) hashes whose
    low word is 0 or 0xFFFFFFFF, which the zeros past s and the padding of
    partial sketches could match by low word: bit-exact against the oracle and
    against the all-checked path (DREPHIP_AP_CMASK=0)."""
    import os
    rng = np.random.default_rng(s + N)
    pool = rng.integers(1, UMAX, size=2 * s, dtype=np.uint64)
    twins = (pool[:s // 8] & np.uint64(0xFFFFFFFF)) | (rng.integers(1, 1 << 32, size=s // 8, dtype=np.uint64)
                                                       << np.uint64(32))
    pool = np.concatenate([pool, twins])
    if edge:
        pool[:4] = (pool[:4] >> np.uint64(32)) << np.uint64(32)                       # low word 0
        pool[4:8] = pool[4:8] | np.uint64(0xFFFFFFFF)                                  # low word 0xFFFFFFFF
    H = np.full((N, s), UMAX, dtype=np.uint64)
    NH = np.zeros(N, dtype=np.uint32)
    for g in range(N):
        vals = np.unique(np.concatenate([rng.choice(pool, size=int(1.2 * s), replace=False),
                                         rng.integers(1, UMAX, size=s // 4, dtype=np.uint64)]))
        n = s if g % 7 else int(rng.integers(1, s))
        NH[g] = min(n, len(vals))
        H[g, :NH[g]] = vals[:NH[g]]
    oc, od = oracle.allpairs(H, NH, s, threads=8)
    os.environ["DREPHIP_SCREEN_MIN_N"] = "2"
    try:
        with _lib.Context(0, 21, s, 42) as ctx:
            c, d = ctx.allpairs(H, NH, want_denom=True)
            st = ctx.screen_stats()
            os.environ["DREPHIP_AP_CMASK"] = "0"
            c0, d0 = ctx.allpairs(H, NH, want_denom=True)
    finally:
        os.environ.pop("DREPHIP_SCREEN_MIN_N")
        os.environ.pop("DREPHIP_AP_CMASK", None)
    assert not st["used"] and st["entries"] == int(NH.sum())          # the screen ran and gave way
    assert np.array_equal(c, oc) and np.array_equal(d, od)
    assert np.array_equal(c0, c) and np.array_equal(d0, d)
    assert (oc > 0).mean() > 0.9


def test_sharded_screen_arguments_checked():
    import torch
    with _lib.Context(0, 21, 1000, 42) as ctx:
        h = torch.zeros((4, 1000), dtype=torch.int64, device="cuda")
        n = torch.zeros(4, dtype=torch.int32, device="cuda")
        with pytest.raises(_lib.DrepHipError, match="part must be below nparts"):
            ctx.screen_part(h.data_ptr(), n.data_ptr(), 4, 2, 2)
        with pytest.raises(_lib.DrepHipError, match="no screen part to copy"):
            ctx.screen_part_copy(h.data_ptr(), h.data_ptr())
        assert ctx.screen_geometry() == 4
