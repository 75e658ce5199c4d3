"""BASELINE configs[2], [3] and [4] in their one-GPU form: 10^4 and 10^5
synthetic 5 Mbp genomes at s = 1000, and 10^4 genomes at s = 10^4 -- sketch,
all-pairs over the whole triangle (5x10^7 / 5x10^9 pairs; 10 GB of condensed
counts in HBM at 10^5) and average-linkage primary clustering (the dense GPU
chain on the n x n float64 matrix, 80 GB at 10^5, built in HBM from the
counts; up to 2x10^4 genomes also the sparse path -- the pairs below 1.0
extracted on the GPU, scipy's chain replayed on them on the host).  All three
run by default.  DREPHIP_SCALE_N=<n> adds one more size (s = 1000).

Parity at full size:
  * the WHOLE triangle against an independent implementation: every pair's
    count is recomputed on the device by k_allpairs_merge (Mash's literal merge
    loop, one lane per pair; oracle-pinned in tests/test_gpu.py) and compared
    with the production kernel's (k_allpairs_q for s <= 2048, k_allpairs_band
    above) -- full_triangle_mismatches must be 0 over all N(N-1)/2 pairs;
  * sketches of a seeded sample of genomes, regenerated and sketched on the
    host by the C oracle, bit-exact;
  * shared-hash counts of random pairs plus three whole rows (first, last,
    random), recomputed by the host oracle's Mash merge from the GPU sketches,
    bit-exact;
  * linkage Z: the sparse and the dense path bit-identical to each other (up
    to 2x10^4 genomes); n-1 merges, monotone heights, consistent sizes; at
    EVERY size bit-identical to scipy's linkage on the host (reference call:
    drep/d_cluster.py:447-457: linkage, then fcluster at 1 - P_ani), and the
    fcluster labels equal.  At 10^5 scipy takes ~2 min and ~80 GB of host
    memory (the 40 GB condensed f64 vector and nn_chain's copy of it).  Z's
    sha1 must also equal the digest committed for the workload in
    tests/golden/scale_linkage_sha1.json (scipy's Z of the same counts).
Timings go to DREPHIP_SCALE_OUT (default gpurun_out/scale_<N>[_s<s>].json).
Reference knobs: MASH_sketch (drep/d_cluster.py:499; CLI -ms,
drep/argumentParser.py:103); Mdb built at drep/d_cluster.py:575-596."""
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
# (genomes, sketch size, BASELINE.json config)
CASES = [pytest.param(1_000, 1000, 100, "BASELINE.json configs[1] (the bench workload)", id="1000"),
         pytest.param(10_000, 1000, 100, "BASELINE.json configs[2] (1 GPU)", id="10000"),
         pytest.param(100_000, 1000, 100, "BASELINE.json configs[3] (1 GPU)", id="100000"),
         pytest.param(10_000, 10_000, 100, "BASELINE.json configs[4] (1 GPU)", id="10000-s10000"),
         # dRep's common job: one species, every pair related (a single family
         # of 10^4 genomes from one ancestor): the screen gives way to the
         # dense kernel; its attempt is timed against the screen forced off
         pytest.param(10_000, 1000, 10_000, "configs[2] size, one species (dense: every pair shares hashes)",
                      id="10000-dense")]
if os.environ.get("DREPHIP_SCALE_N"):
    _n = int(os.environ["DREPHIP_SCALE_N"])
    CASES.append(pytest.param(_n, int(os.environ.get("DREPHIP_SCALE_S", 1000)),
                              int(os.environ.get("DREPHIP_SCALE_FAM", 100)), "custom", id="custom%d" % _n))
if os.environ.get("DREPHIP_SCALE_ONLY"):
    CASES = [c for c in CASES if c.id in os.environ["DREPHIP_SCALE_ONLY"].split(",")]
# scipy's Z digest per workload (test id), committed after a run in which Z
# equalled scipy's (the result JSON records it as linkage_sha1)
DIGESTS = os.path.join(ROOT, "tests", "golden", "scale_linkage_sha1.json")


def z_digest(Z):
    import hashlib
    return hashlib.sha1(np.ascontiguousarray(Z, dtype="<f8").tobytes()).hexdigest()


def _cond_index(i, j, N):
    i = i.astype(np.int64)
    j = j.astype(np.int64)
    return i * N - i * (i + 1) // 2 + (j - i - 1)


def full_triangle_check(ctx, hh, nn, N, d_common, note, parts=16):
    """Every pair of the triangle recomputed by k_allpairs_merge (Mash's
    literal loop) and compared on the device; row ranges of ~equal pair count,
    so progress is reported while the (slower) literal kernel runs.  Returns
    (mismatches, seconds, examples)."""
    import torch
    from drep_amd.parallel import cond_start, row_partition, segment_size
    dev = d_common.device
    stream = torch.cuda.current_stream(dev).cuda_stream
    bad, ex = 0, []
    t0 = time.perf_counter()
    for r0, r1 in row_partition(N, parts):
        n = segment_size(N, r0, r1)
        if n == 0:
            continue
        a = cond_start(r0, N)
        b = a + n
        seg = torch.empty(n, dtype=torch.int16, device=dev)
        ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, r0, r1, seg.data_ptr(), None, stream, merge=True)
        ne = d_common[a:b] != seg
        nb = int(ne.sum().item())
        if nb and len(ex) < 20:
            w = torch.nonzero(ne)[:20 - len(ex), 0].cpu().numpy() + a
            ex += [[int(t), int(d_common[t].item()), int(seg[t - a].item())] for t in w]
        bad += nb
        del seg, ne
        note("full triangle: rows [%d, %d) checked, %d mismatches so far (%.1f s)"
             % (r0, r1, bad, time.perf_counter() - t0))
    torch.cuda.synchronize()
    return bad, time.perf_counter() - t0, ex


@pytest.mark.parametrize("N,s,fam,config", CASES)
@pytest.mark.timeout(900)
def test_scale(N, s, fam, config):
    import torch
    L = int(os.environ.get("DREPHIP_SCALE_L", 5_000_000))
    seed = 0xD2E9
    CH = min(N, int(os.environ.get("DREPHIP_SCALE_CHUNK", 10000)))
    out_path = os.environ.get("DREPHIP_SCALE_OUT", os.path.join(
        ROOT, "gpurun_out", "scale_%d%s%s.json" % (N, "" if s == 1000 else "_s%d" % s, "" if fam == 100 else "_dense")))
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    log = open(os.path.splitext(out_path)[0] + ".progress", "a")

    def note(msg):
        line = "%.1f %s" % (time.time(), msg)
        print(line, flush=True)
        log.write(line + "\n")
        log.flush()

    res = {"genomes": N, "genome_bp": L, "sketch": s, "family_size": fam, "pairs": N * (N - 1) // 2,
           "config": config}
    dev = torch.device("cuda", 0)
    ctx = _lib.Context(device=0, k=21, s=s, seed=42)
    stream = torch.cuda.current_stream(dev).cuda_stream
    # the n x n linkage matrix (80 GB at 10^5, ~2 s of hipMalloc) is allocated
    # by the clustering context on a helper thread while the sketch and
    # all-pairs stages run (as drep_amd.distributed does on its root rank)
    import threading
    link_ctx = _lib.Context(device=0, k=21, s=s, seed=42)
    reserve_t = {}

    def reserve():
        t0 = time.perf_counter()
        link_ctx.linkage_reserve(N)
        reserve_t["s"] = time.perf_counter() - t0
    reserver = threading.Thread(target=reserve, daemon=True)
    reserver.start()

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
    ctx.set_timing(True, kernels=[2, 4])                 # the all-pairs kernels and the screen (HIP events)
    t0 = time.perf_counter()
    ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, 0, N, d_common.data_ptr(), None, stream)
    torch.cuda.synchronize()
    res["allpairs_s"] = time.perf_counter() - t0
    res["allpairs_pairs_per_s"] = npairs / res["allpairs_s"]
    res["allpairs_screen"] = ctx.screen_stats()
    res["allpairs_screen_ms"] = ctx.kernel_ms(4)[0]
    res["allpairs_kernel_ms"] = ctx.kernel_ms(2)[0]
    note("allpairs %.3f s (%.3g pairs/s) screen %s (%.2f ms) kernel %.2f ms"
         % (res["allpairs_s"], res["allpairs_pairs_per_s"], json.dumps(res["allpairs_screen"]),
            res["allpairs_screen_ms"], res["allpairs_kernel_ms"]))
    if fam != 100:
        # the same call with the screen off: what the screen's attempt (runs
        # counted, then given way to the dense kernel) costs on a dense set
        d2 = torch.zeros(npairs, dtype=torch.int16, device=dev)
        ctx.set_allpairs_screen(ctx.SCREEN_OFF)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, 0, N, d2.data_ptr(), None, stream)
            torch.cuda.synchronize()
        res["allpairs_screen_off_s"] = time.perf_counter() - t0
        res["allpairs_screen_off_kernel_ms"] = ctx.kernel_ms(2)[0]
        res["allpairs_screen_off_pairs_per_s"] = npairs / res["allpairs_screen_off_s"]
        res["dense_kernel_pairs_per_s"] = npairs / (res["allpairs_screen_off_kernel_ms"] * 1e-3)
        ctx.set_allpairs_screen(ctx.SCREEN_AUTO)
        assert bool((d2 == d_common).all().item())
        # and again in auto mode, warm: the screen's attempt before it gives way
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, 0, N, d2.data_ptr(), None, stream)
        torch.cuda.synchronize()
        res["allpairs_auto_warm_s"] = time.perf_counter() - t0
        res["allpairs_auto_warm_screen_ms"] = ctx.kernel_ms(4)[0]
        res["allpairs_auto_warm_kernel_ms"] = ctx.kernel_ms(2)[0]
        note("dense set: screen off %.3f s (kernel %.2f ms, %.3g pairs/s); auto (warm) %.3f s, screen attempt %.2f ms"
             % (res["allpairs_screen_off_s"], res["allpairs_screen_off_kernel_ms"], res["dense_kernel_pairs_per_s"],
                res["allpairs_auto_warm_s"], res["allpairs_auto_warm_screen_ms"]))
        del d2
    ctx.set_timing(False)

    # ---- parity: the whole triangle against the literal-merge kernel
    nbad, t_full, ex = full_triangle_check(ctx, hh, nn, N, d_common, note)
    res["full_triangle_pairs"] = npairs
    res["full_triangle_mismatches"] = nbad
    res["full_triangle_check_s"] = t_full
    res["full_triangle_checker"] = "k_allpairs_merge (Mash's literal merge loop, one lane per pair)"
    if nbad:
        res["full_triangle_mismatch_examples"] = ex
        json.dump(res, open(out_path, "w"), indent=1)
    torch.cuda.empty_cache()
    assert nbad == 0

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
    M = 1_000_000 if s <= 2048 else 100_000      # host merge cost grows with s
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
    t0 = time.perf_counter()
    reserver.join()
    res["linkage_reserve_s"] = reserve_t.get("s")              # on the helper thread, beside the stages above
    res["linkage_reserve_wait_s"] = time.perf_counter() - t0
    link_ctx.set_timing(True)
    # the automatic path (dense here: at s = 1000 random shared hashes join the
    # families into one component), then -- up to 2x10^4 genomes -- the sparse
    # path forced (the pairs below 1.0 extracted on the GPU, scipy's chain
    # replayed on them on the host): two independent implementations,
    # compared bit for bit
    t0 = time.perf_counter()
    Z = link_ctx.linkage_counts_device(d_common.data_ptr(), None, N, perm, lut, lut_off, "average", stream)
    res["linkage_s"] = time.perf_counter() - t0
    res["linkage_info"] = link_ctx.linkage_info()
    res["linkage_matrix_build_ms"] = link_ctx.kernel_ms(3)[0]
    res["linkage_chain_ms"] = link_ctx.kernel_ms(2)[0]
    res["linkage_phases_s"] = link_ctx.linkage_stats()
    res["linkage_chain_launches"] = link_ctx.linkage_launches()
    res["linkage_launches_per_merge"] = res["linkage_chain_launches"] / (N - 1)
    note("linkage (%s) %.3f s %s %s (matrix reserved in %.2f s beside sketch/all-pairs, waited %.3f s)"
         % ("sparse" if res["linkage_info"]["sparse"] else "dense", res["linkage_s"],
            json.dumps(res["linkage_phases_s"]), json.dumps(res["linkage_info"]),
            res["linkage_reserve_s"] or -1, res["linkage_reserve_wait_s"]))
    if N <= 20_000:
        link_ctx.set_linkage_path(link_ctx.LINK_DENSE if res["linkage_info"]["sparse"] else link_ctx.LINK_SPARSE)
        t0 = time.perf_counter()
        Z2 = link_ctx.linkage_counts_device(d_common.data_ptr(), None, N, perm, lut, lut_off, "average", stream)
        other = "sparse" if link_ctx.linkage_info()["sparse"] else "dense"
        res["linkage_%s_s" % other] = time.perf_counter() - t0
        res["linkage_%s_phases_s" % other] = link_ctx.linkage_stats()
        res["linkage_sparse_equals_dense"] = bool(np.array_equal(Z, Z2))
        note("linkage (%s) %.3f s %s; sparse == dense: %s" % (other, res["linkage_%s_s" % other],
                                                            json.dumps(link_ctx.linkage_stats()),
                                                            res["linkage_sparse_equals_dense"]))
        assert res["linkage_sparse_equals_dense"]
    assert Z.shape == (N - 1, 4)
    assert np.all(np.diff(Z[:, 2]) >= 0)           # average linkage is monotone
    assert Z[-1, 3] == N
    assert np.all(Z[:, 0] < Z[:, 1])
    import scipy.cluster.hierarchy as sch
    fcl = sch.fcluster(Z, 0.1, criterion="distance")
    res["primary_clusters_at_P_ani_0.9"] = int(fcl.max())
    res["linkage_sha1"] = z_digest(Z)
    case = ("%d" % N if s == 1000 else "%d-s%d" % (N, s)) + ("" if fam == 100 else "-dense")
    golden = json.load(open(DIGESTS)).get(case) if os.path.exists(DIGESTS) else None
    res["linkage_sha1_golden"] = golden
    note("Z sha1 %s (golden %s)" % (res["linkage_sha1"], golden))
    json.dump(res, open(out_path, "w"), indent=1)

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
    res["scipy_linkage_sha1"] = z_digest(Zs)
    fcl_s = sch.fcluster(Zs, 0.1, criterion="distance")
    res["fcluster_labels_identical_to_scipy"] = bool(np.array_equal(fcl, fcl_s))
    del y, Zs
    note("scipy linkage %.1f s identical=%s, fcluster labels identical=%s"
         % (res["scipy_linkage_s"], res["linkage_identical_to_scipy"], res["fcluster_labels_identical_to_scipy"]))
    json.dump(res, open(out_path, "w"), indent=1)
    assert res["linkage_identical_to_scipy"]
    assert res["fcluster_labels_identical_to_scipy"]
    if golden is not None:
        assert res["linkage_sha1"] == golden
    link_ctx.close()
    ctx.close()
    json.dump(res, open(out_path, "w"), indent=1)
    note(json.dumps(res))
