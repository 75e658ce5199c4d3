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


def _run(world, out, port):
    env = dict(os.environ, DREPHIP_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "drep_amd.distributed",
           "--genomes", str(N), "--genome-bp", str(L), "--family-size", "20", "--out", out]
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
    for world, port in ((2, 29621), (3, 29631)):
        res = _run(world, str(tmp_path / ("w%d" % world)), port)
        assert res["n_gpus"] == world
        cm = load_condensed(str(tmp_path / ("w%d" % world)), mmap=False)
        pl = load_primary_linkage(str(tmp_path / ("w%d" % world)))
        cdb = pd.read_csv(tmp_path / ("w%d" % world) / "primary_Cdb.csv")
        assert np.array_equal(cm.common, cm1.common)
        assert np.array_equal(pl["linkage"], pl1["linkage"])
        assert cdb.equals(cdb1)
