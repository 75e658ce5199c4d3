"""BASELINE configs[2] and configs[3] in their one-GPU form: 10^4 and 10^5
synthetic 5 Mbp genomes, s = 1000 -- sketch, all-pairs over the whole triangle
(5x10^7 / 5x10^9 pairs; 10 GB of condensed counts in HBM at 10^5) and
average-linkage primary clustering on the GPU (the n x n float64 matrix, 80 GB
at 10^5, built in HBM from the counts).  Both sizes run by default; the
GPU time is seconds (sketch 0.9 s, all-pairs 1.1 s, linkage 2.3 s at 10^5).
DREPHIP_SCALE_N=<n> adds one more size.

Parity at full size, through what the oracle can afford:
  * sketches of a seeded sample of genomes, regenerated and sketched on the
    host by the C oracle, bit-exact;
  * shared-hash counts of 10^6 random pairs plus three whole rows (first,
    last, random), recomputed by the oracle's Mash merge from the GPU sketches,
    bit-exact;
  * a second all-pairs pass over the same sketches: identical triangle;
  * linkage Z: n-1 merges, monotone heights, consistent sizes; at 10^4 also
    bit-identical to scipy's linkage on the host (reference call:
    drep/d_cluster.py:453; ~1 s of host time).  At 10^5 the scipy comparison
    (121 s of host time) runs only with DREPHIP_SCALE_SCIPY=1.
Timings go to DREPHIP_SCALE_OUT (default gpurun_out/scale_<N>.json)."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import oracle
from drep_amd import _lib
from drep_amd.d_cluster import linkage_tables

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = [10_000, 100_000]
if os.environ.get("DREPHIP_SCALE_N"):
    SIZES.append(int(os.environ["DREPHIP_SCALE_N"]))
SCIPY_UP_TO = 10_000 if os.environ.get("DREPHIP_SCALE_SCIPY") != "1" else 10 ** 9


def _cond_index(i, j, N):
    i = i.astype(np.int64)
    j = j.astype(np.int64)
    return i * N - i * (i + 1) // 2 + (j - i - 1)


@pytest.mark.parametrize("N", SIZES)
@pytest.mark.timeout(600)
def test_scale_sketch_allpairs_linkage_single_gpu(N):
    import torch
    L = int(os.environ.get("DREPHIP_SCALE_L", 5_000_000))
    s = 1000
    fam = 100
    seed = 0xD2E9
    CH = min(N, int(os.environ.get("DREPHIP_SCALE_CHUNK", 10000)))
    out_path = os.environ.get("DREPHIP_SCALE_OUT", os.path.join(ROOT, "gpurun_out", "scale_%d.json" % N))
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    log = open(os.path.splitext(out_path)[0] + ".progress", "a")

    def note(msg):
        line = "%.1f %s" % (time.time(), msg)
        print(line, flush=True)
        log.write(line + "\n")
        log.flush()

    res = {"genomes": N, "genome_bp": L, "sketch": s, "family_size": fam, "pairs": N * (N - 1) // 2,
           "config": {10_000: "BASELINE.json configs[2] (1 GPU)", 100_000: "BASELINE.json configs[3] (1 GPU)"}
           .get(N, "custom")}
    dev = torch.device("cuda", 0)
    ctx = _lib.Context(device=0, k=21, s=s, seed=42)
    stream = torch.cuda.current_stream(dev).cuda_stream

    # ---- sketch, CH genomes at a time (inputs generated on device, untimed)
    tile = _lib.tile_bases()
    P = _lib.padded_bases([L])
    total = tile + CH * P
    codes = torch.zeros(total // 16, dtype=torch.int32, device=dev)
    valid = torch.zeros(total // 32, dtype=torch.int32, device=dev)
    hh = torch.full((N, s), -1, dtype=torch.int64, device=dev)
    nn = torch.zeros(N, dtype=torch.int32, device=dev)
    t_sketch = 0.0
    for g0 in range(0, N, CH):
        n = min(CH, N - g0)
        ctx.synth_device(seed, g0, n, fam, L, codes.data_ptr(), valid.data_ptr(), stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.sketch_device(codes.data_ptr(), valid.data_ptr(), np.array([tile + i * P for i in range(n)], np.uint64),
                          np.full(n, P, np.uint64), np.full(n, L - 20, np.uint64), n,
                          hh[g0].data_ptr(), nn[g0:].data_ptr(), stream)
        torch.cuda.synchronize()
        t_sketch += time.perf_counter() - t0
        note("sketched %d/%d" % (g0 + n, N))
    del codes, valid
    torch.cuda.empty_cache()
    res["sketch_s"] = t_sketch
    res["sketch_GBps_ascii"] = N * L / t_sketch / 1e9

    # ---- all-pairs over the whole triangle
    npairs = N * (N - 1) // 2
    d_common = torch.zeros(npairs, dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, 0, N, d_common.data_ptr(), None, stream)
    torch.cuda.synchronize()
    res["allpairs_s"] = time.perf_counter() - t0
    res["allpairs_pairs_per_s"] = npairs / res["allpairs_s"]
    note("allpairs %.3f s (%.3g pairs/s)" % (res["allpairs_s"], res["allpairs_pairs_per_s"]))
    # idempotence: a second pass over the same sketches gives the same triangle
    d_again = torch.zeros(npairs, dtype=torch.int16, device=dev)
    ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, 0, N, d_again.data_ptr(), None, stream)
    torch.cuda.synchronize()
    ndiff = int((d_again != d_common).sum().item())
    res["second_pass_differences"] = ndiff
    del d_again
    torch.cuda.empty_cache()
    note("second pass differences: %d" % ndiff)
    assert ndiff == 0

    # ---- parity: sketches of sampled genomes (host oracle regenerates the genome)
    H = hh.cpu().numpy().view(np.uint64)
    NH = nn.cpu().numpy().view(np.uint32)
    assert (NH == s).all()
    rng = np.random.default_rng(N)
    threads = min(16, oracle.max_threads())
    g_blk = int(rng.integers(0, N - threads))
    ref_h, ref_n = oracle.sketch_synth(g_blk, threads, L, seed=seed, family_size=fam, s=s, threads=threads)
    assert np.array_equal(H[g_blk:g_blk + threads], ref_h) and (ref_n == s).all()
    for g in (0, N - 1):
        rh, _ = oracle.sketch_synth(g, 1, L, seed=seed, family_size=fam, s=s, threads=1)
        assert np.array_equal(H[g], rh[0]), g
    res["sketch_parity_genomes"] = threads + 2
    note("sketch parity ok")

    # ---- parity: counts of random pairs and of whole rows, recomputed by the oracle
    M = 1_000_000
    pi = rng.integers(0, N - 1, M)
    pj = pi + 1 + (rng.random(M) * (N - 1 - pi)).astype(np.int64)
    for r in (0, N - 2, int(rng.integers(1, N - 2))):
        pi = np.concatenate([pi, np.full(N - 1 - r, r)])
        pj = np.concatenate([pj, np.arange(r + 1, N)])
    idx = torch.from_numpy(_cond_index(pi, pj, N)).to(dev)
    got = d_common[idx].cpu().numpy().view(np.uint16)
    want = oracle.dist_pairs_list(H, NH, s, pi, pj, threads=threads)
    bad = np.nonzero(got != want)[0]
    if len(bad):
        res["pair_mismatches"] = int(len(bad))
        res["pair_mismatch_examples"] = [[int(pi[b]), int(pj[b]), int(got[b]), int(want[b])] for b in bad[:40]]
        json.dump(res, open(out_path, "w"), indent=1)
    assert len(bad) == 0
    res["pair_parity_pairs"] = int(len(pi))
    res["common_histogram_sample"] = np.bincount(got, minlength=s + 1)[[0, 1, 10, 100, 500, 1000]].tolist()
    note("pair parity ok (%d pairs)" % len(pi))
    del hh, nn, idx
    torch.cuda.empty_cache()

    # ---- primary clustering: average linkage on the GPU from the device counts
    lut, lut_off = linkage_tables(np.array([s]), s)
    perm = np.arange(N, dtype=np.uint32)          # names g000000.. sort in index order
    ctx.set_timing(True)
    t0 = time.perf_counter()
    Z = ctx.linkage_counts_device(d_common.data_ptr(), None, N, perm, lut, lut_off, "average")
    res["linkage_s"] = time.perf_counter() - t0
    res["linkage_matrix_build_ms"] = ctx.kernel_ms(3)[0]
    res["linkage_chain_ms"] = ctx.kernel_ms(2)[0]
    note("gpu linkage %.2f s" % res["linkage_s"])
    assert Z.shape == (N - 1, 4)
    assert np.all(np.diff(Z[:, 2]) >= 0)           # average linkage is monotone
    assert Z[-1, 3] == N
    assert np.all(Z[:, 0] < Z[:, 1])
    import scipy.cluster.hierarchy as sch
    fcl = sch.fcluster(Z, 0.1, criterion="distance")
    res["primary_clusters_at_P_ani_0.9"] = int(fcl.max())

    if N <= SCIPY_UP_TO:
        common = d_common.cpu().numpy().view(np.uint16)
        del d_common
        torch.cuda.empty_cache()
        y = np.empty(npairs, dtype=np.float64)
        step = 1 << 27
        for a in range(0, npairs, step):
            y[a:a + step] = lut[common[a:a + step]]
        del common
        hb = subprocess.Popen([sys.executable, "-c",
                               "import time,sys\nwhile True:\n print(time.time(), 'scipy linkage running', "
                               "file=open(sys.argv[1], 'a'), flush=True); time.sleep(20)",
                               os.path.splitext(out_path)[0] + ".progress"])
        try:
            t0 = time.perf_counter()
            Zs = sch.linkage(y, method="average")
            res["scipy_linkage_s"] = time.perf_counter() - t0
        finally:
            hb.kill()
            hb.wait()
        res["linkage_identical_to_scipy"] = bool(np.array_equal(Z, Zs))
        note("scipy linkage %.1f s identical=%s" % (res["scipy_linkage_s"], res["linkage_identical_to_scipy"]))
        assert res["linkage_identical_to_scipy"]
    ctx.close()
    json.dump(res, open(out_path, "w"), indent=1)
    note(json.dumps(res))
