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
            if N >= 1000:
                assert max(sizes) - min(sizes) <= N          # within one row


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
