"""The sharded configs[3] job (python -m drep_amd.distributed under
torch.distributed.run) rehearsed on one MI355X: 2 and 3 ranks share the GPU
over gloo (segments staged through the host; the 8-GPU run uses RCCL), and
the root's stored condensed counts, linkage and primary Cdb must equal the
1-rank job's and the oracle's sampled counts."""
import json
import os
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

import oracle
from drep_amd.store import load_condensed, load_primary_linkage

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, L = 240, 300_000


def _run(world, out, port, n=N, sketch=1000, screen=None, shard=None):
    # the root's condensed vector starts poisoned: every pair must be written
    env = dict(os.environ, DREPHIP_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1", DREPHIP_SEGMENT_POISON="1")
    if screen is not None:          # the shared-hash screen forced on (1) / off (2) in every rank
        env["DREPHIP_AP_SCREEN"] = str(screen)
    if shard is not None:           # the sharded screen (default on) / every rank grouping all entries
        env["DREPHIP_SCREEN_SHARD"] = str(shard)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "drep_amd.distributed",
           "--genomes", str(n), "--genome-bp", str(L), "--family-size", "20", "--sketch", str(sketch),
           "--out", out]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.timeout(600)
def test_sharded_job_matches_single_rank(tmp_path):
    one = _run(1, str(tmp_path / "w1"), 29611)
    cm1 = load_condensed(str(tmp_path / "w1"), mmap=False)
    pl1 = load_primary_linkage(str(tmp_path / "w1"))
    cdb1 = pd.read_csv(tmp_path / "w1" / "primary_Cdb.csv")
    assert pl1["arguments"]["linkage_method"] == "average" and pl1["db"] is None
    assert one["primary_clusters"] > 1
    # counts: a sample against the oracle's merge of the oracle's sketches
    h, nh = oracle.sketch_synth(0, N, L, seed=0xD2E9, family_size=20, threads=8)
    assert np.array_equal(cm1.nhash, nh)
    want, _ = oracle.allpairs(h, nh, 1000, r0=0, r1=12, threads=8)
    assert np.array_equal(cm1.common[:len(want)], want)
    # world 8 as the driver's 8-GPU run has it (8 gloo ranks sharing this GPU):
    # every partition edge of row_partition / genome_shard at 8 ranks
    for world, port in ((2, 29621), (3, 29631), (8, 29711)):
        res = _run(world, str(tmp_path / ("w%d" % world)), port)
        assert res["n_gpus"] == world
        cm = load_condensed(str(tmp_path / ("w%d" % world)), mmap=False)
        pl = load_primary_linkage(str(tmp_path / ("w%d" % world)))
        cdb = pd.read_csv(tmp_path / ("w%d" % world) / "primary_Cdb.csv")
        assert np.array_equal(cm.common, cm1.common)
        assert np.array_equal(pl["linkage"], pl1["linkage"])
        assert cdb.equals(cdb1)


@pytest.mark.timeout(600)
def test_sharded_job_band_path_matches_single_rank(tmp_path):
    """s = 4096 (> 2048: the value-band kernel, configs[4]'s path): the root's
    segment written in place into its slice of the full vector (out=), the
    other rank's received into its slice; the vector starts poisoned and no
    pair may keep the poison.  1 and 2 ranks give the same counts, Z and Cdb,
    and rows of the counts equal the oracle's merge."""
    n, s = 96, 4096
    one = _run(1, str(tmp_path / "b1"), 29661, n=n, sketch=s, screen=2)
    two = _run(2, str(tmp_path / "b2"), 29671, n=n, sketch=s, screen=2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    cm1 = load_condensed(str(tmp_path / "b1"), mmap=False)
    cm2 = load_condensed(str(tmp_path / "b2"), mmap=False)
    assert np.array_equal(cm1.common, cm2.common)
    assert np.array_equal(load_primary_linkage(str(tmp_path / "b1"))["linkage"],
                          load_primary_linkage(str(tmp_path / "b2"))["linkage"])
    assert pd.read_csv(tmp_path / "b1" / "primary_Cdb.csv").equals(pd.read_csv(tmp_path / "b2" / "primary_Cdb.csv"))
    h, nh = oracle.sketch_synth(0, n, L, seed=0xD2E9, family_size=20, s=s, threads=8)
    assert np.array_equal(cm1.nhash, nh)
    # the first rows (rank 0's in-place segment) and the last rows (rank 1's)
    for r0, r1 in ((0, 4), (n - 6, n - 1)):
        want, _ = oracle.allpairs(h, nh, s, r0=r0, r1=r1, threads=8)
        a = r0 * n - r0 * (r0 + 1) // 2
        assert np.array_equal(cm2.common[a:a + len(want)], want), (r0, r1)
    # the same with the shared-hash screen forced on in both ranks: the
    # no-shared-hash fill plus the LIST band kernel write every pair
    three = _run(2, str(tmp_path / "b3"), 29681, n=n, sketch=s, screen=1)
    assert three["n_gpus"] == 2
    cm3 = load_condensed(str(tmp_path / "b3"), mmap=False)
    assert np.array_equal(cm3.common, cm1.common)
    assert np.array_equal(load_primary_linkage(str(tmp_path / "b3"))["linkage"],
                          load_primary_linkage(str(tmp_path / "b1"))["linkage"])


@pytest.mark.timeout(600)
def test_sharded_job_screened_matches_unscreened(tmp_path):
    """s = 1000 (whole-row kernel): 3 and 8 ranks with the shared-hash screen
    forced on -- sharded by hash range (each rank groups one part, the marks
    exchanged), and at 3 ranks also unsharded (every rank groups every entry)
    -- equal 1 rank with it off (stored counts, Z, Cdb), the root's vector
    starting poisoned."""
    off = _run(1, str(tmp_path / "off"), 29691, screen=2)
    assert off["n_gpus"] == 1
    a = load_condensed(str(tmp_path / "off"), mmap=False)
    for name, world, port, shard in (("on", 3, 29701, None), ("on8", 8, 29721, None), ("flat", 3, 29731, 0)):
        on = _run(world, str(tmp_path / name), port, screen=1, shard=shard)
        assert on["n_gpus"] == world
        b = load_condensed(str(tmp_path / name), mmap=False)
        assert np.array_equal(a.common, b.common), name
        assert np.array_equal(load_primary_linkage(str(tmp_path / "off"))["linkage"],
                              load_primary_linkage(str(tmp_path / name))["linkage"]), name
        assert pd.read_csv(tmp_path / "off" / "primary_Cdb.csv").equals(pd.read_csv(tmp_path / name / "primary_Cdb.csv"))


def _file_set(tmp_path, copies=6):
    """The 4 reference FASTAs, each copied under `copies` distinct names, plus
    Sakai as a location whose FASTA is absent and whose sketch is cached in the
    work directory (as in the reference's own test work directory)."""
    import shutil
    golden = os.path.join(ROOT, "tests", "golden")
    gdir = tmp_path / "genomes"
    gdir.mkdir()
    locs = []
    for k in range(copies):
        for fa in sorted(os.listdir(os.path.join(golden, "genomes"))):
            dst = gdir / ("c%d_%s" % (k, fa))
            shutil.copy(os.path.join(golden, "genomes", fa), dst)
            locs.append(str(dst))
    locs.append(str(gdir / "Escherichia_coli_Sakai.fna"))
    sakai = os.path.join(golden, "MASH_files", "sketches", "Escherichia_coli_Sakai.fna.msh")

    def data_folder(name):
        d = tmp_path / name
        chunk = d / "MASH_files" / "sketches" / "chunk_0"
        chunk.mkdir(parents=True)
        shutil.copy(sakai, chunk / "Escherichia_coli_Sakai.fna.msh")
        return str(d)
    return locs, data_folder


@pytest.mark.timeout(600)
def test_sharded_job_on_files_matches_drop_in(tmp_path):
    """`drep_amd.distributed --files` (2 ranks sharing the GPU over gloo) on
    real FASTA files plus a cached sketch: stored counts, Z and Cdb equal the
    single-process drop-in's all_vs_all_MASH_condensed + cluster_mash_condensed
    (reference path: d_cluster.py:527-549 sketch stage, 170-185 clustering)."""
    import pandas as pd
    from drep_amd.d_cluster import all_vs_all_MASH_condensed, cluster_mash_condensed
    locs, data_folder = _file_set(tmp_path)
    lst = tmp_path / "genomes.txt"
    lst.write_text("\n".join(locs) + "\n")
    Bdb = pd.DataFrame({"genome": [os.path.basename(x) for x in locs], "location": locs})
    cm = all_vs_all_MASH_condensed(Bdb, data_folder("wd_single"), processors=4)
    Cdb, (Z, _, _) = cluster_mash_condensed(cm, clusterAlg="average", P_ani=0.9)
    assert int(cm.nhash[-1]) == 1000 and len(set(Cdb["primary_cluster"])) > 1
    for world, port in ((2, 29641), (1, 29651)):
        out = str(tmp_path / ("out%d" % world))
        env = dict(os.environ, DREPHIP_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "drep_amd.distributed",
               "--files", str(lst), "--data-folder", data_folder("wd_dist%d" % world), "--processors", "4",
               "--out", out]
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-3000:]
        res = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
        assert res["input"] == "files (1 cached sketches)" and res["genomes"] == len(locs)
        cmd_ = load_condensed(out, mmap=False)
        pl = load_primary_linkage(out)
        cdb = pd.read_csv(os.path.join(out, "primary_Cdb.csv"))
        assert cmd_.names == cm.names and cmd_.locations == cm.locations
        assert np.array_equal(cmd_.common, cm.common) and np.array_equal(cmd_.nhash, cm.nhash)
        assert np.array_equal(cmd_.length, cm.length)
        assert np.array_equal(pl["linkage"], Z)
        assert np.array_equal(cdb["primary_cluster"].to_numpy(), Cdb["primary_cluster"].to_numpy())
        assert list(cdb["genome"]) == list(Cdb["genome"])


def _uneven_file_set(tmp_path):
    """FASTAs of very different lengths: each reference genome alone and
    concatenated with 1-3 others as one multi-record file (~2.5-12 Mbp)."""
    import gzip
    golden = os.path.join(ROOT, "tests", "golden", "genomes")
    fas = sorted(os.listdir(golden))
    raw = [gzip.open(os.path.join(golden, f)).read() for f in fas]
    gdir = tmp_path / "uneven"
    gdir.mkdir()
    locs = []
    for k in range(10):
        parts = [raw[(k + j) % len(raw)] for j in range(1 + (k * 7) % 4)]
        dst = gdir / ("u%02d.fna" % k)
        dst.write_bytes(b"".join(p if p.endswith(b"\n") else p + b"\n" for p in parts))
        locs.append(str(dst))
    return locs


@pytest.mark.timeout(600)
def test_sharded_job_balanced_file_shards_match_drop_in(tmp_path):
    """--files with genomes of very different lengths: the sketch shards are
    balanced by file size (parallel.balanced_shards), the
    per-rank byte totals within one file of each other, and the stored names,
    counts, lengths, Z and Cdb equal the single-process drop-in's
    (reference: d_cluster.py:527-549 sketch fan-out, 170-185 clustering)."""
    from drep_amd.d_cluster import all_vs_all_MASH_condensed, cluster_mash_condensed
    locs = _uneven_file_set(tmp_path)
    sizes = [os.path.getsize(x) for x in locs]
    assert max(sizes) > 3 * min(sizes)
    lst = tmp_path / "uneven.txt"
    lst.write_text("\n".join(locs) + "\n")
    Bdb = pd.DataFrame({"genome": [os.path.basename(x) for x in locs], "location": locs})
    wd = tmp_path / "wd_single"
    wd.mkdir()
    cm = all_vs_all_MASH_condensed(Bdb, str(wd), processors=4)
    Cdb, (Z, _, _) = cluster_mash_condensed(cm, clusterAlg="average", P_ani=0.9)
    for world, port in ((3, 29721), (2, 29731)):
        out = str(tmp_path / ("uout%d" % world))
        env = dict(os.environ, DREPHIP_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "drep_amd.distributed",
               "--files", str(lst), "--processors", "4", "--out", out]
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-3000:]
        res = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
        w = res["shard_weights"]
        assert len(w) == world and max(w) - min(w) <= max(sizes)
        got = load_condensed(out, mmap=False)
        assert got.names == cm.names and got.locations == cm.locations
        assert np.array_equal(got.common, cm.common) and np.array_equal(got.nhash, cm.nhash)
        assert np.array_equal(got.length, cm.length)
        assert np.array_equal(load_primary_linkage(out)["linkage"], Z)
        cdb = pd.read_csv(os.path.join(out, "primary_Cdb.csv"))
        assert list(cdb["genome"]) == list(Cdb["genome"])
        assert np.array_equal(cdb["primary_cluster"].to_numpy(), Cdb["primary_cluster"].to_numpy())
