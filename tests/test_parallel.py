"""Multi-rank sharding on CPU with gloo (world size 2 and 3): genome shards ->
all-gather -> balanced row shards -> reassembled condensed triangle equals the
single-process result.  The per-rank compute is the oracle here (no GPU); the
plumbing is the same code bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest

from drep_amd import parallel

S = 300


def test_row_partition_balanced_and_covering():
    for N in (2, 3, 10, 1000, 10001):
        for W in (1, 2, 3, 8):
            parts = parallel.row_partition(N, W)
            assert parts[0][0] == 0 and parts[-1][1] == N
            assert all(a[1] == b[0] for a, b in zip(parts[:-1], parts[1:]))
            sizes = [parallel.segment_size(N, a, b) for a, b in parts]
            assert sum(sizes) == N * (N - 1) // 2
            assert all(a % parallel.ROW_ALIGN == 0 for a, _ in parts[1:] if a < N)   # tile-aligned
            if N >= 1000:
                # within one row of balance, up to the alignment (ROW_ALIGN rows)
                assert max(sizes) - min(sizes) <= 2 * parallel.ROW_ALIGN * N


def test_genome_shards_cover():
    for N in (1, 5, 1000, 1001):
        for W in (1, 2, 8):
            got = []
            for r in range(W):
                g0, g1, nmax = parallel.genome_shard(N, W, r)
                assert g1 - g0 <= nmax
                got += list(range(g0, g1))
            assert got == list(range(N))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, out_dir):
    import torch
    import torch.distributed as dist
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g0, g1, nmax = parallel.genome_shard(N, world, rank)
    h, nh = oracle.sketch_synth(g0, g1 - g0, 60_000, seed=4, family_size=5, s=S, threads=1)
    loc_h = torch.full((nmax, S), -1, dtype=torch.int64)
    loc_n = torch.zeros(nmax, dtype=torch.int32)
    loc_h[:g1 - g0] = torch.from_numpy(h.view(np.int64))
    loc_n[:g1 - g0] = torch.from_numpy(nh.view(np.int32))
    all_h, all_n = parallel.gather_sketches(loc_h, loc_n)
    H = all_h[:N].numpy().view(np.uint64)
    NH = all_n[:N].numpy().view(np.uint32)
    r0, r1 = parallel.row_partition(N, world)[rank]
    seg, _ = oracle.allpairs(H, NH, S, r0=r0, r1=min(r1, N - 1) if r0 < N - 1 else r0, threads=1)
    np.save(os.path.join(out_dir, "seg%d.npy" % rank), seg[:parallel.segment_size(N, r0, r1)])
    np.save(os.path.join(out_dir, "H%d.npy" % rank), H)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_pipeline_matches_single_process(tmp_path, world):
    import torch.multiprocessing as mp
    import oracle
    N = 23
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, N, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    segs = [np.load(os.path.join(tmp_path, "seg%d.npy" % r)) for r in range(world)]
    full = parallel.assemble_condensed(N, segs, world)
    h, nh = oracle.sketch_synth(0, N, 60_000, seed=4, family_size=5, s=S, threads=2)
    want, _ = oracle.allpairs(h, nh, S)
    assert np.array_equal(full, want)
    for r in range(world):   # every rank saw the full, ordered sketch matrix
        assert np.array_equal(np.load(os.path.join(tmp_path, "H%d.npy" % r)), h)


def _worker_pipeline(rank, world, port, N, out_dir, partial):
    """One rank of drep_amd.distributed.run_sharded with CPU stand-ins for the
    HIP stages (oracle sketch / merge, scipy linkage): the sharding, the
    all-gather, the uneven segment gather to the root and the root's
    clustering are the product code."""
    import torch
    import torch.distributed as dist
    import oracle
    from drep_amd import distributed as D
    from drep_amd.d_cluster import CondensedMash, cluster_mash_condensed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    names = D.synthetic_names(N)

    def sketch_fn(p):
        loc_h = torch.full((p.nmax, S), -1, dtype=torch.int64)
        loc_n = torch.zeros(p.nmax, dtype=torch.int32)
        if p.g1 > p.g0:
            h, nh = oracle.sketch_synth(p.g0, p.g1 - p.g0, 60_000, seed=4, family_size=5, s=S, threads=1)
            if partial:                      # genomes 5, 6, 7 keep a partial sketch
                for g in range(p.g0, p.g1):
                    if g in (5, 6, 7):
                        h[g - p.g0, 100 + g:] = np.iinfo(np.uint64).max
                        nh[g - p.g0] = 100 + g
            loc_h[:p.g1 - p.g0] = torch.from_numpy(h.view(np.int64))
            loc_n[:p.g1 - p.g0] = torch.from_numpy(nh.view(np.int32))
        return loc_h, loc_n

    def allpairs_fn(H, NH, p, out=None):
        Hn = H.numpy().view(np.uint64)
        Nn = NH.numpy().view(np.uint32)
        if not p.seg_len:
            return torch.zeros(1, dtype=torch.int16), torch.zeros(1, dtype=torch.int16)
        c, d = oracle.allpairs(Hn, Nn, S, r0=p.r0, r1=min(p.r1, N - 1), threads=1)
        return (torch.from_numpy(c[:p.seg_len].view(np.int16).copy()),
                torch.from_numpy(d[:p.seg_len].view(np.int16).copy()))

    def linkage_fn(common, denom, n, method):
        c = common.numpy().view(np.uint16)
        d = denom.numpy().view(np.uint16) if denom is not None else np.full(len(c), S, np.uint16)
        cm = CondensedMash(names, names, c, d, np.zeros(n, np.uint32), np.zeros(n, np.uint64), S)
        _, (Z, _, _) = cluster_mash_condensed(cm, clusterAlg=method, gpu=None)
        return Z

    res = D.run_sharded(N, names, S, sketch_fn, allpairs_fn, linkage_fn, "average", 0.9)
    if rank == 0:
        np.save(os.path.join(out_dir, "Z.npy"), res["linkage"])
        np.save(os.path.join(out_dir, "common.npy"), res["common"].numpy().view(np.uint16))
        if res["denom"] is not None:
            np.save(os.path.join(out_dir, "denom.npy"), res["denom"].numpy().view(np.uint16))
        res["Cdb"].to_csv(os.path.join(out_dir, "Cdb.csv"), index=False)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,partial", [(2, False), (3, False), (3, True)])
def test_gloo_sharded_clustering_matches_single_process(tmp_path, world, partial):
    """configs[3]'s sharded job (drep_amd.distributed.run_sharded) on CPU with
    gloo: the root's reassembled condensed counts, linkage Z and primary Cdb
    equal the single-process result (reference chain d_cluster.py:170-185)."""
    import pandas as pd
    import torch.multiprocessing as mp
    import oracle
    from drep_amd import distributed as D
    from drep_amd.d_cluster import CondensedMash, cluster_mash_condensed
    N = 29
    port = _free_port()
    mp.start_processes(_worker_pipeline, args=(world, port, N, str(tmp_path), partial), nprocs=world, join=True,
                       start_method="spawn")
    h, nh = oracle.sketch_synth(0, N, 60_000, seed=4, family_size=5, s=S, threads=2)
    if partial:
        for g in (5, 6, 7):
            h[g, 100 + g:] = np.iinfo(np.uint64).max
            nh[g] = 100 + g
    want_c, want_d = oracle.allpairs(h, nh, S)
    assert np.array_equal(np.load(os.path.join(tmp_path, "common.npy")), want_c)
    if partial:
        assert np.array_equal(np.load(os.path.join(tmp_path, "denom.npy")), want_d)
        assert (want_d < S).any()
    names = D.synthetic_names(N)
    cm = CondensedMash(names, names, want_c, want_d, nh, np.zeros(N, np.uint64), S)
    cdb, (Z, _, _) = cluster_mash_condensed(cm, clusterAlg="average", P_ani=0.9, gpu=None)
    assert np.array_equal(np.load(os.path.join(tmp_path, "Z.npy")), Z)
    got = pd.read_csv(os.path.join(tmp_path, "Cdb.csv"))
    assert got["genome"].tolist() == cdb["genome"].tolist()
    assert got["primary_cluster"].tolist() == cdb["primary_cluster"].tolist()
    assert cdb["primary_cluster"].nunique() > 1


def test_shard_plan_covers_everything():
    from drep_amd import distributed as D
    for N in (2, 7, 1000, 100_000):
        for W in (1, 2, 3, 8):
            ps = [D.plan(N, W, r) for r in range(W)]
            assert sum(p.seg_len for p in ps) == N * (N - 1) // 2
            assert sum(p.g1 - p.g0 for p in ps) == N
            for a, b in zip(ps[:-1], ps[1:]):
                assert a.seg0 + a.seg_len == b.seg0 or b.seg_len == 0


def test_balanced_shards_by_weight():
    """sketch shards balanced greedily by bases; every rank's
    total within one genome's weight of every other's, every genome once."""
    rng = np.random.default_rng(5)
    for N in (1, 5, 29, 1000):
        for W in (1, 2, 3, 8):
            w = rng.integers(1, 10_000_000, N).astype(np.float64)
            w[rng.random(N) < 0.1] = 0            # cached sketches weigh nothing
            sh = parallel.balanced_shards(w, W)
            got = np.sort(np.concatenate(sh))
            assert np.array_equal(got, np.arange(N))
            tot = np.array([w[m].sum() for m in sh])
            assert tot.max() - tot.min() <= w.max()
            nmax, pos = parallel.shard_layout(sh, N)
            assert nmax == max(1, max(len(m) for m in sh))
            for r, m in enumerate(sh):
                assert np.array_equal(pos[m], r * nmax + np.arange(len(m)))


def test_balanced_shards_zero_weights_spread():
    """A rerun with every sketch cached weighs every genome 0: the shards must
    still be of near-equal count (the all-gather pads to the largest)."""
    for N in (1, 7, 100, 1001):
        for W in (1, 2, 3, 8):
            sh = parallel.balanced_shards(np.zeros(N), W)
            assert max(len(m) for m in sh) == -(-N // W)
            nmax, _ = parallel.shard_layout(sh, N)
            assert nmax == max(1, -(-N // W))
            # mostly cached: the few real genomes balance, the rest fill up evenly
            w = np.zeros(N)
            w[: max(1, N // 50)] = 5e6
            sh = parallel.balanced_shards(w, W)
            assert max(len(m) for m in sh) - min(len(m) for m in sh) <= 1


def _len_of(g):
    # genome lengths spread over 20x (5 kbp .. 100 kbp): a count split would be badly unbalanced
    return 5_000 + (g * 37_813) % 95_000


def _worker_weighted(rank, world, port, N, out_dir):
    """run_sharded with balanced shards (weights = genome lengths): each rank
    sketches a non-contiguous set of genomes; the gathered rows must come back
    in genome order."""
    import torch
    import torch.distributed as dist
    import oracle
    from drep_amd import distributed as D
    from drep_amd.d_cluster import CondensedMash, cluster_mash_condensed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    names = D.synthetic_names(N)
    weights = [float(_len_of(g)) for g in range(N)]

    def sketch_fn(p):
        assert p.pos is not None and p.g0 == -1
        loc_h = torch.full((p.nmax, S), -1, dtype=torch.int64)
        loc_n = torch.zeros(p.nmax, dtype=torch.int32)
        for j, g in enumerate(p.genomes()):
            h, nh = oracle.sketch_synth(int(g), 1, _len_of(int(g)), seed=4, family_size=5, s=S, threads=1)
            loc_h[j] = torch.from_numpy(h[0].view(np.int64))
            loc_n[j] = int(nh[0])
        np.save(os.path.join(out_dir, "members%d.npy" % rank), p.genomes())
        return loc_h, loc_n

    def allpairs_fn(H, NH, p, out=None):
        Hn = H.numpy().view(np.uint64)
        Nn = NH.numpy().view(np.uint32)
        if not p.seg_len:
            return torch.zeros(1, dtype=torch.int16), torch.zeros(1, dtype=torch.int16)
        c, d = oracle.allpairs(Hn, Nn, S, r0=p.r0, r1=min(p.r1, N - 1), threads=1)
        return (torch.from_numpy(c[:p.seg_len].view(np.int16).copy()),
                torch.from_numpy(d[:p.seg_len].view(np.int16).copy()))

    def linkage_fn(common, denom, n, method):
        c = common.numpy().view(np.uint16)
        d = denom.numpy().view(np.uint16) if denom is not None else np.full(len(c), S, np.uint16)
        cm = CondensedMash(names, names, c, d, np.zeros(n, np.uint32), np.zeros(n, np.uint64), S)
        _, (Z, _, _) = cluster_mash_condensed(cm, clusterAlg=method, gpu=None)
        return Z

    res = D.run_sharded(N, names, S, sketch_fn, allpairs_fn, linkage_fn, "average", 0.9, weights=weights)
    if rank == 0:
        np.save(os.path.join(out_dir, "Z.npy"), res["linkage"])
        np.save(os.path.join(out_dir, "common.npy"), res["common"].numpy().view(np.uint16))
        np.save(os.path.join(out_dir, "H.npy"), res["hashes"].numpy().view(np.uint64))
        res["Cdb"].to_csv(os.path.join(out_dir, "Cdb.csv"), index=False)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_balanced_shards_match_single_process(tmp_path, world):
    """Genomes of very different lengths, sketch shards balanced by length:
    per-rank totals within one genome of each other; the root's sketch matrix
    (genome order), counts, Z and Cdb equal the single-process result."""
    import pandas as pd
    import torch.multiprocessing as mp
    import oracle
    from drep_amd import distributed as D
    from drep_amd.d_cluster import CondensedMash, cluster_mash_condensed
    N = 31
    port = _free_port()
    mp.start_processes(_worker_weighted, args=(world, port, N, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    mem = [np.load(os.path.join(tmp_path, "members%d.npy" % r)) for r in range(world)]
    lens = np.array([_len_of(g) for g in range(N)])
    tot = [lens[m].sum() for m in mem]
    assert max(tot) - min(tot) <= lens.max()
    assert not all(np.array_equal(m, np.arange(m[0], m[-1] + 1)) for m in mem if len(m))   # not contiguous
    h = np.full((N, S), np.iinfo(np.uint64).max, dtype=np.uint64)
    nh = np.zeros(N, dtype=np.uint32)
    for g in range(N):
        hg, ng = oracle.sketch_synth(g, 1, _len_of(g), seed=4, family_size=5, s=S, threads=1)
        h[g], nh[g] = hg[0], ng[0]
    assert np.array_equal(np.load(os.path.join(tmp_path, "H.npy")), h)
    want_c, want_d = oracle.allpairs(h, nh, S)
    assert np.array_equal(np.load(os.path.join(tmp_path, "common.npy")), want_c)
    names = D.synthetic_names(N)
    cm = CondensedMash(names, names, want_c, want_d, nh, np.zeros(N, np.uint64), S)
    cdb, (Z, _, _) = cluster_mash_condensed(cm, clusterAlg="average", P_ani=0.9, gpu=None)
    assert np.array_equal(np.load(os.path.join(tmp_path, "Z.npy")), Z)
    got = pd.read_csv(os.path.join(tmp_path, "Cdb.csv"))
    assert got["genome"].tolist() == cdb["genome"].tolist()
    assert got["primary_cluster"].tolist() == cdb["primary_cluster"].tolist()


def test_file_weights(tmp_path):
    import gzip
    from drep_amd import distributed as D
    a = tmp_path / "a.fa"
    a.write_bytes(b">x\n" + b"ACGT" * 1000 + b"\n")
    b = tmp_path / "b.fa.gz"
    with gzip.open(b, "wb") as f:
        f.write(b">y\n" + b"A" * 50_000 + b"\n")
    w = D.file_weights([str(a), str(b), str(tmp_path / "missing.fa"), str(a)], cached={3: object()})
    assert w[0] == os.path.getsize(a)
    assert w[1] == 50_000 + 4               # the gzip trailer's uncompressed size
    assert w[2] == 0 and w[3] == 0           # unreadable; cached


def test_file_weights_multi_member_and_bgzf(tmp_path):
    """The gzip trailer only holds the last member's size: a bgzip file (last
    member empty, ISIZE 0) and a multi-member file whose last member is small
    are estimated from the compressed size instead of being under-counted."""
    import gzip
    import random
    import struct
    import zlib
    from drep_amd import distributed as D
    rnd = random.Random(3)
    seq = b">z\n" + bytes(rnd.choice(b"ACGT") for _ in range(200_000)) + b"\n"
    multi = tmp_path / "m.fa.gz"
    multi.write_bytes(gzip.compress(seq) + gzip.compress(b">t\nAC\n"))
    size = os.path.getsize(multi)
    assert D.file_weights([str(multi)])[0] == size * D.GZIP_DNA_RATIO

    def bgzf_block(data):
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        cdata = co.compress(data) + co.flush()
        bsize = 18 + len(cdata) + 8 - 1
        hdr = b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<H", 6) + b"BC" + struct.pack("<HH", 2, bsize)
        return hdr + cdata + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))
    bg = tmp_path / "b.fa.gz"
    bg.write_bytes(bgzf_block(seq[:60_000]) + bgzf_block(seq[60_000:]) + bgzf_block(b""))
    assert gzip.decompress(bg.read_bytes()) == seq
    assert D.file_weights([str(bg)])[0] == os.path.getsize(bg) * D.GZIP_DNA_RATIO
    single = tmp_path / "s.fa.gz"
    single.write_bytes(gzip.compress(seq))
    assert D.file_weights([str(single)])[0] == len(seq)


def _xworker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    starts, R = _xstarts(world), 4
    rng = np.random.default_rng(rank)
    nc, nr = 6 + 2 * rank, (rank * 2) % 3                  # one part sends no records
    T = rng.integers(0, 10 * world // R + 1, nc)
    cells = np.stack([T, rng.integers(0, 9, nc), np.full(nc, rank), np.arange(nc)], 1).astype(np.int32)
    a = rng.integers(0, 10 * world, nr)
    recs = np.stack([a, a + 1, np.full(nr, rank), np.arange(nr)], 1).astype(np.int32)
    # buffers longer than the counts (rows past them are ignored)
    cpad = torch.from_numpy(np.concatenate([cells, np.full((2, 4), -7, np.int32)]))
    rpad = torch.from_numpy(np.concatenate([recs, np.full((1, 4), -7, np.int32)]))
    got_c, got_r, checks = parallel.exchange_screen_parts(cpad, nc, rpad, nr, 10 ** rank, starts, R)
    np.save(os.path.join(out_dir, "c%d.npy" % rank), got_c.numpy())
    np.save(os.path.join(out_dir, "r%d.npy" % rank), got_r.numpy())
    np.save(os.path.join(out_dir, "sc%d.npy" % rank), cells)
    np.save(os.path.join(out_dir, "sr%d.npy" % rank), recs)
    np.save(os.path.join(out_dir, "k%d.npy" % rank), np.array([checks]))
    dist.destroy_process_group()


def _xstarts(world):
    starts = [10 * r for r in range(world)]
    if world > 2:
        starts[2] = starts[1]                              # rank 1's rows empty
    return starts


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange_screen_parts(tmp_path, world):
    """The sharded screen's exchange (parallel.exchange_screen_parts): every
    cell word lands on the rank owning its row tile's first row, every record
    on the rank owning its row a, in source-part order, with an empty part and
    a rank without rows; the pair checks summed."""
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_xworker, args=(world, port, str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    starts = _xstarts(world)
    sc = np.concatenate([np.load(os.path.join(tmp_path, "sc%d.npy" % r)) for r in range(world)])
    sr = np.concatenate([np.load(os.path.join(tmp_path, "sr%d.npy" % r)) for r in range(world)])
    oc = np.searchsorted(starts, sc[:, 0] * 4, side="right") - 1
    orr = np.searchsorted(starts, sr[:, 0], side="right") - 1
    for r in range(world):
        gc = np.load(os.path.join(tmp_path, "c%d.npy" % r))
        gr = np.load(os.path.join(tmp_path, "r%d.npy" % r))
        wc, wr = sc[oc == r], sr[orr == r]
        assert np.array_equal(gc, wc[np.lexsort((wc[:, 3], wc[:, 2]))]), r
        assert np.array_equal(gr.reshape(-1, 4), wr[np.lexsort((wr[:, 3], wr[:, 2]))]), r
        assert int(np.load(os.path.join(tmp_path, "k%d.npy" % r))[0]) == sum(10 ** q for q in range(world))
