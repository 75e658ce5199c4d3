#!/usr/bin/env python3
"""Benchmark of the dRep primary-clustering hot path on MI355X.

One *step* = one pass of the hot path over the synthetic genome set, inputs
already resident in HBM (2-bit packed, generated on device):
  1. sketch every genome of this rank's shard  (replaces `mash sketch`, d_cluster.py:543)
  2. RCCL all-gather of the sketch shards       (replaces `mash paste`,  d_cluster.py:551-567)
  3. all-pairs shared-hash counts for this rank's balanced row range of the
     upper triangle                             (replaces `mash dist`,   d_cluster.py:570-573)
value = N(N-1)/2 genome pairs / step time, whole job (all ranks; max over ranks).

Default workload = BASELINE.json configs[1]: 1,000 synthetic 5 Mbp genomes,
k=21, s=1000.  The same total workload is used at every GPU count (strong
scaling).  Launch: `python bench.py` (1 GPU), `python bench.py --gpus N`
(starts N ranks itself, one per GPU, under torch.distributed.run as a child
process) or `python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N`.

Two throughputs: `value` is the whole step (sketch + exchange + all-pairs),
end to end; `dist_pairs_per_s` is the metric's own quantity per SURVEY.md
§8(d): pairs / all-pairs stage time with the sketches resident.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU issue: MI355X_MICROARCH.md gives one wave64 VALU instruction per 2
# cycles per SIMD (SIMD-32) as the issue peak: 1024 SIMDs x 2.4 GHz / 2 (the
# all-pairs kernel's VALU fraction is quoted against it).  The sketch hash
# kernel's peak is its priced instruction stream (profiles/r06_sketch_priced.json,
# tools/sketch_priced.py): every instruction of the hot loop at its class's
# measured wall time per wave64 instruction per SIMD with 8 waves on every SIMD
# (tools/valu_microbench.hip) -- full-rate classes ~1.0 ns, the 64-bit,
# multiply, 3-operand and byte-select classes ~1.75 ns.
N_SIMD = 256 * 4
VALU_PEAK_WAVE_INST = N_SIMD * 2.4e9 / 2
SKETCH_PHASES = os.path.join(ROOT, "profiles", "r05_sketch_isa_phases.json")
SKETCH_PRICED = os.path.join(ROOT, "profiles", "r06_sketch_priced.json")
# Committed rocprofv3 summaries this line quotes.  A profile carries the
# library build it was taken on (drephip_build_id, "build_id") and the
# workload; the line quotes one only when both are this run's -- a profile of
# another build or workload is named in a note, never used for a fraction.
#   sketch: tools/profile_round.sh (traffic_json.py / pmc_summary.py)
#   all-pairs: tools/profile_allpairs.sh (allpairs_traffic_json.py), one file
#   per workload: rNN_allpairs_N<N>_s<s>_f<family size>.json, newest round first
PROFILES = os.path.join(ROOT, "profiles")
SKETCH_PMC_NAME = "sketch_pmc_sq.json"
SKETCH_TRAFFIC_NAME = "sketch_traffic.json"
PROFILE_STEPS = 3              # untimed steps that time finalize / all-pairs / table build
VERIFY_GENOMES = 16            # timed-step sketches re-derived by the C oracle (sampled, every run)
VERIFY_PAIRS = 100_000         # timed-step counts re-derived by the C oracle (random pairs + one row)


def lib_build_src():
    from drep_amd import _lib
    return _lib.build_id().get("src")


def find_profile(name, accept=None):
    """The newest profiles/rNN_<name> taken on THIS library build (and, given
    `accept`, whose content it accepts).  Returns (doc, path, note): doc None
    when no such profile exists, with the reason in `note`."""
    import glob
    import re
    src = lib_build_src()
    cands = sorted(glob.glob(os.path.join(PROFILES, "r[0-9][0-9]_" + name)),
                   key=lambda p: int(re.search(r"/r(\d\d)_", p).group(1)), reverse=True)
    seen = []
    for path in cands:
        try:
            d = json.load(open(path))
        except Exception:
            continue
        rel = os.path.relpath(path, ROOT)
        b = (d.get("build_id") or {}).get("src")
        if b != src:
            seen.append("%s: build %s" % (rel, (b or "unrecorded")[:12]))
            continue
        if accept is not None and not accept(d):
            seen.append("%s: another workload/kernel" % rel)
            continue
        return d, rel, None
    return None, None, ("no profiles/rNN_%s of this library build (src %s)%s" %
                        (name, (src or "?")[:12], ("; not used: " + "; ".join(seen)) if seen else ""))


def dist_roofline(N, s, fam, screened, pairs_per_launch, launch_ms):
    """Roofline block of the all-pairs kernel this run used -- the dense
    k_allpairs_q / k_allpairs_band template, or the screened LIST one -- from
    the committed profile of exactly this workload (N, s, family size) and
    kernel template on this library build (tools/profile_allpairs.sh): VALU
    issue against the 2-cycle wave64 peak (the PMC's VALU instructions per pair
    x this launch's pairs / this launch's live HIP-event time), LDS busy, HBM
    traffic against the algorithmic bytes and the L2 hit rate of the profiled
    dispatches.  No matching profile: no fraction, only the reason."""
    variant = "LIST" if screened else "dense"

    def accept(d):
        w = d.get("workload") or {}
        return (w.get("genomes"), w.get("sketch"), w.get("family_size"), w.get("kernel_variant")) == (N, s, fam, variant)
    d, rel, note = find_profile("allpairs_N%d_s%d_f%d.json" % (N, s, fam), accept)
    if d is None:
        return {"kernel_variant": variant, "note": note}
    dv = d.get("derived", {})
    out = {"kernel": (d.get("kernel") or "")[:60], "kernel_variant": variant, "source": rel,
           "build_id": d["build_id"].get("src"), "profiled_avg_call_ms": d.get("avg_call_ms"),
           "this_run_ms": launch_ms}
    if dv.get("valu_wave_insts_per_pair") and launch_ms and not screened:
        ach = dv["valu_wave_insts_per_pair"] * pairs_per_launch / (launch_ms * 1e-3)
        out.update({"bound": "valu+salu+lds (co-bound, DESIGN.md 10)", "achieved": ach, "peak": VALU_PEAK_WAVE_INST,
                    "unit": "wave64 VALU instructions/s", "frac": ach / VALU_PEAK_WAVE_INST,
                    "valu_wave_insts_per_pair": dv["valu_wave_insts_per_pair"],
                    "salu_over_valu": dv.get("salu_over_valu")})
        salu = (d.get("counters_per_call") or {}).get("SQ_INSTS_SALU")
        if salu and dv.get("kernel_cycles"):
            # one scalar unit per CU issues at most one instruction per cycle
            out["salu_per_cu_cycle"] = salu / (256.0 * dv["kernel_cycles"])
    for k in ("lds_busy_frac", "lds_bank_conflict_frac", "valu_issue_frac_2cyc", "wait_inst_any_frac",
              "wait_any_frac", "l2_hit_rate", "hbm_bytes_x2", "hbm_GBps_x2", "hbm_frac_of_8TBps_x2",
              "algorithmic_bytes", "hbm_over_algorithmic_x2", "effective_clock_ghz", "pairs_per_s"):
        if k in dv:
            out[k] = dv[k]
    out["traffic"] = dv.get("hbm_bytes_x2")
    return out


def pmc_block(doc, rel):
    """Utilisation fractions from a committed PMC summary, or None."""
    if doc is None:
        return None
    # (valu_active_quad_frac is not kept: SQ_ACTIVE_INST_VALU equals
    # SQ_INSTS_VALU in the sketch profile, i.e. it counts one quad-cycle per
    # instruction, so that "fraction" is the instruction count priced at 4
    # cycles, not a measured VALU occupancy)
    keep = ("valu_issue_frac_2cyc", "lds_busy_frac", "lds_bank_conflict_frac", "wait_any_frac",
            "wait_inst_any_frac", "active_inst_any_frac", "valu_insts_per_window_end", "effective_clock_ghz")
    out = {k: doc["derived"][k] for k in keep if k in doc.get("derived", {})}
    out["source"] = rel
    out["build_id"] = (doc.get("build_id") or {}).get("src")
    out["profiled_kernel"] = (doc.get("kernel") or "")[:80]
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--genomes", type=int, default=1000)
    ap.add_argument("--genome-bp", type=int, default=5_000_000)
    ap.add_argument("--sketch", type=int, default=1000)
    ap.add_argument("--family-size", type=int, default=100)
    ap.add_argument("--seed", type=int, default=0xD2E9)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the C oracle on host cores (rank 0)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="queue each step before checking the previous one (1) or one step at a time (0)")
    ap.add_argument("--defer-check", type=int, default=1,
                    help="check the sketch's threshold status after queuing the all-pairs (1) or before (0)")
    ap.add_argument("--check", type=int, default=1,
                    help="after timing (untimed): check a sample of the timed steps' own sketches and "
                         "shared-hash counts against the C oracle (test infrastructure); 'verified' in "
                         "the JSON line")
    ap.add_argument("--verify", type=int, default=0,
                    help="after timing, every rank re-sketches all genomes and recomputes the whole "
                         "triangle on its own GPU and checks its gathered sketches and its segment "
                         "(rehearsal of the sharded path; untimed)")
    return ap.parse_args()


def config_name(N, L, s):
    """Which BASELINE.json config a run measures (the default is configs[1])."""
    if L == 5_000_000:
        if (N, s) == (1000, 1000):
            return "BASELINE.json configs[1]"
        if (N, s) == (10000, 1000):
            return "BASELINE.json configs[2]"
        if (N, s) == (100000, 1000):
            return "BASELINE.json configs[3]"
        if (N, s) == (10000, 10000):
            return "BASELINE.json configs[4]"
    return "custom size"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(args, threads, share):
    """The same whole job on the host with the C oracle (Mash-equivalent
    restatement, OpenMP): sketch every genome and `mash dist` every pair when
    that fits CPU_BUDGET_S of wall time (configs[1]: ~19 s on the GPU box's 16
    threads), else a bounded sample extrapolated to the job: a probe of
    16 x threads genomes sketched first decides which."""
    import oracle
    N, L, s = args.genomes, args.genome_bp, args.sketch
    budget = float(os.environ.get("CPU_BUDGET_S", 30))
    ns = min(N, max(2, 16 * threads))
    t0 = time.perf_counter()
    h, nh = oracle.sketch_synth(0, ns, L, seed=args.seed, family_size=args.family_size, s=s, threads=threads)
    t_sk = time.perf_counter() - t0
    if ns < N and t_sk / ns * N <= budget:                       # the whole sketch fits: measure it
        t0 = time.perf_counter()
        h2, nh2 = oracle.sketch_synth(ns, N - ns, L, seed=args.seed, family_size=args.family_size, s=s,
                                      threads=threads)
        t_sk += time.perf_counter() - t0
        h, nh = np.concatenate([h, h2]), np.concatenate([nh, nh2])
        ns = N
    full = ns == N and N * (N - 1) // 2 <= 5_000_000
    if full:                                                     # every pair of the job
        iu = np.triu_indices(N, 1)
        pi, pj = iu[0].astype(np.uint32), iu[1].astype(np.uint32)
    else:                                                        # random pairs of the sampled genomes
        rng = np.random.default_rng(1)
        npairs = max(2, min(N * (N - 1) // 2, 5_000_000))
        pi = rng.integers(0, ns, npairs).astype(np.uint32)
        pj = ((pi + 1 + rng.integers(0, ns - 1, npairs)) % ns).astype(np.uint32)
    npairs = len(pi)
    t0 = time.perf_counter()
    oracle.dist_pairs_list(h, nh, s, pi, pj, threads=threads)
    t_d = time.perf_counter() - t0
    per_genome = t_sk / ns
    per_pair = t_d / npairs
    job = N * per_genome + (N * (N - 1) / 2) * per_pair
    visible = share["visible_cpus"] or threads
    if ns == N and full:
        how = ("the whole job measured: sketch of all %d synthetic %d bp genomes in %.2f s + all %d pairs of "
               "mash dist in %.2f s" % (N, L, t_sk, npairs, t_d))
    else:
        how = ("sketch of %d of the %d synthetic %d bp genomes in %.2f s + %d pairs of mash dist in %.2f s; job = "
               "%d x per-genome sketch + N(N-1)/2 x per-pair dist = %.1f s + %.2f s"
               % (ns, N, L, t_sk, npairs, t_d, N, N * per_genome, N * (N - 1) / 2 * per_pair))
    out = {
        "value": (N * (N - 1) / 2) / job,
        "unit": "genome pairs/s",
        "cores": threads,
        "kind": "port",
        "cpu_model": cpu_model(),
        "host_cpus_visible": visible,
        "sample": "C oracle (Mash-equivalent restatement; Mash itself is absent), OpenMP on all %d host CPUs "
                  "this job may use (mash dist -p <all host cores>, d_cluster.py:570); %s" % (threads, how),
        "host_cpu_share": share,
        "measured_whole_job": bool(ns == N and full),
        "sketch_Mbp_per_s": ns * L / t_sk / 1e6,
        "dist_pairs_per_s": npairs / t_d,
    }
    if visible > threads:
        # the machine has more CPUs than this job may use: the measured rate
        # scaled linearly to all of them, labelled as an extrapolation
        out["value_all_visible_cpus_extrapolated"] = (N * (N - 1) / 2) / job * visible / threads
        out["extrapolation_note"] = ("%d of %d visible CPUs are this job's share; linear scaling assumed"
                                     % (threads, visible))
    return out


def check_against_oracle(args, loc_h, loc_n, d_common, g0, nloc, N, r0, r1, world, gather_sketches):
    """Sampled check of the timed steps' outputs (untimed; the C oracle is test
    infrastructure): VERIFY_GENOMES of this rank's genomes regenerated and
    sketched on the host must equal their rows of the sketch matrix, and the
    shared-hash counts of VERIFY_PAIRS random pairs of this rank's segment plus
    one whole row must equal Mash's merge of the gathered sketches."""
    import torch
    import oracle
    from drep_amd.parallel import cond_start, segment_size
    L, s = args.genome_bp, args.sketch
    threads = max(1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1))
    rng = np.random.default_rng(12345 + g0)
    res = {"genomes": 0, "pairs": 0, "mismatches": 0}
    ok = True
    if nloc:
        k = min(VERIFY_GENOMES, nloc)
        starts = sorted(set([0, nloc - 1] + [int(x) for x in rng.integers(0, nloc, k - 2)])) if k > 2 else list(range(k))
        H = loc_h[:nloc].cpu().numpy().view(np.uint64)
        NH = loc_n[:nloc].cpu().numpy().view(np.uint32)
        for i in starts:
            oh, onh = oracle.sketch_synth(g0 + i, 1, L, seed=args.seed, family_size=args.family_size, s=s,
                                          threads=threads)
            good = bool(np.array_equal(H[i], oh[0]) and NH[i] == onh[0])
            ok &= good
            res["mismatches"] += int(not good)
        res["genomes"] = len(starts)
    seg = segment_size(N, r0, r1)
    # the gather is a collective: every rank joins it, also one whose segment
    # is empty (row_partition may give the last rank no pairs at small N)
    hh, nn = (gather_sketches(loc_h, loc_n) if world > 1 else (loc_h, loc_n))
    if seg:
        HA = hh[:N].cpu().numpy().view(np.uint64)
        NA = nn[:N].cpu().numpy().view(np.uint32)
        C = d_common[:seg].cpu().numpy().view(np.uint16)
        a = cond_start(r0, N)
        t = rng.integers(0, seg, VERIFY_PAIRS) + a                     # condensed indices in this segment
        row = int(rng.integers(r0, min(r1, N - 1)))                    # plus one whole row
        t = np.concatenate([t, cond_start(row, N) + np.arange(N - 1 - row)])
        # condensed index -> (i, j)
        Mf = 2.0 * N - 1.0
        i = np.floor((Mf - np.sqrt(np.maximum(Mf * Mf - 8.0 * t, 0.0))) / 2.0).astype(np.int64)
        i = np.clip(i, 0, N - 2)
        for _ in range(2):
            i = np.where(i * N - i * (i + 1) // 2 > t, i - 1, i)
            i = np.where((i + 1) * N - (i + 1) * (i + 2) // 2 <= t, i + 1, i)
        j = t - (i * N - i * (i + 1) // 2) + i + 1
        want = oracle.dist_pairs_list(HA, NA, s, i.astype(np.uint32), j.astype(np.uint32), threads=threads)
        bad = int((C[t - a] != want).sum())
        ok &= bad == 0
        res["pairs"] = int(len(t))
        res["mismatches"] += bad
    if world > 1:
        import torch.distributed as dist
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=loc_h.device)
        tot = torch.tensor([res["genomes"], res["pairs"], res["mismatches"]], dtype=torch.int64,
                           device=loc_h.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        ok = bool(flag.item())
        res.update(genomes=int(tot[0].item()), pairs=int(tot[1].item()), mismatches=int(tot[2].item()))
    res["verified"] = bool(ok)
    return res


def launch_ranks(args):
    """`--gpus N` without torch.distributed.run around us: start N ranks (one
    per GPU) as a child `python -m torch.distributed.run` on 127.0.0.1 -- a
    child process, started before this process touches the GPU -- and return
    its exit code.  Rank 0 prints the JSON line to the inherited stdout."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print("bench: starting %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    # rank 0's JSON line goes to stdout; anything else the ranks print there
    # (gloo's connection messages) is relayed to stderr
    p = subprocess.Popen(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"), stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return p.wait()


def host_cpu_share():
    """The host CPUs this job may use: the CPU affinity mask, capped by a
    cgroup v2 CPU quota (cpu.max) and by OMP_NUM_THREADS when either is set
    (the GPU box gives a one-GPU job 16 of the visible CPUs)."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    cores = aff
    if quota:
        cores = min(cores, max(1, math.floor(quota)))
    if omp:
        cores = min(cores, omp)
    return cores, {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "omp_num_threads": omp,
                   "visible_cpus": os.cpu_count()}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        print("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        return 2
    import torch
    import torch.distributed as dist
    backend = os.environ.get("DREPHIP_DIST_BACKEND", "nccl")          # nccl = RCCL over xGMI
    if world > 1 and backend == "nccl" and world > torch.cuda.device_count():
        # RCCL needs one GPU per rank (gloo may share one, for rehearsals)
        print("bench: %d ranks over RCCL but %d GPUs visible" % (world, torch.cuda.device_count()), file=sys.stderr)
        return 2
    # one rank per GPU; ranks beyond the visible GPUs wrap (only for rehearsing
    # the multi-rank path on a smaller box, with DREPHIP_DIST_BACKEND=gloo)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from drep_amd import _lib
    from drep_amd.parallel import cond_start, genome_shard, row_partition, segment_size, gather_sketches

    N, L, s = args.genomes, args.genome_bp, args.sketch
    ctx = _lib.Context(device=local, k=21, s=s, seed=42)
    # the timed steps bracket only the dominant kernel (sketch hash) with HIP
    # events: every event pair leaves an idle gap of several microseconds
    # between dispatches; the other kernels are timed in extra steps afterwards
    ctx.set_timing(True, kernels=(0,))
    dev = torch.device("cuda", local)
    # every library call runs on torch's stream, so it is ordered after the
    # tensor fills / all-gathers that torch issues there
    stream = torch.cuda.current_stream(dev).cuda_stream

    # ---- this rank's genome shard, generated on device (untimed)
    g0, g1, nmax = genome_shard(N, world, rank)
    nloc = g1 - g0
    tile = _lib.tile_bases()
    P = _lib.padded_bases([L])
    total_bases = tile + max(nloc, 1) * P
    codes = torch.zeros(total_bases // 16, dtype=torch.int32, device=dev)
    valid = torch.zeros(total_bases // 32, dtype=torch.int32, device=dev)
    if nloc:
        ctx.synth_device(args.seed, g0, nloc, args.family_size, L, codes.data_ptr(), valid.data_ptr(), stream)
    base_off = np.array([tile + i * P for i in range(nloc)], np.uint64)
    padded = np.full(nloc, P, np.uint64)
    nkmers = np.full(nloc, L - 20, np.uint64)
    loc_h = torch.full((nmax, s), -1, dtype=torch.int64, device=dev)
    loc_n = torch.zeros(nmax, dtype=torch.int32, device=dev)
    r0, r1 = row_partition(N, world)[rank]
    seg = segment_size(N, r0, r1)
    d_common = torch.zeros(max(seg, 1), dtype=torch.int16, device=dev)
    # several ranks with the screen on (N >= 4096): the screen sharded by hash
    # range, its marks exchanged (every rank calls it, synchronous)
    from drep_amd.distributed import allpairs_rows_sharded, sharded_screen_applies
    sharded = sharded_screen_applies(ctx, N)

    def allpairs_sharded(hh, nn):
        return allpairs_rows_sharded(ctx, hh, nn, N, r0, r1, d_common.data_ptr() if seg else None, None, stream, dev)

    stage = {"sketch": 0.0, "gather": 0.0, "dist": 0.0}
    kms = {0: [0.0, 0], 1: [0.0, 0], 2: [0.0, 0], 3: [0.0, 0], 4: [0.0, 0]}

    ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]

    redo = {"n": 0}

    def read_kms(which):
        for w in which:
            ms, n = ctx.kernel_ms(w)
            kms[w][0] += ms
            kms[w][1] += n

    def step(record):
        if nloc:
            # the sketch's threshold-round status is checked after the all-pairs
            # call (sketch_wait), so the gather and all-pairs queue right behind
            # the sketch kernels without a host round trip in between
            sketch = ctx.sketch_device_async if args.defer_check else ctx.sketch_device
            sketch(codes.data_ptr(), valid.data_ptr(), base_off, padded, nkmers, nloc,
                   loc_h.data_ptr(), loc_n.data_ptr(), stream)
            if record and not args.defer_check:
                read_kms((0, 1))
        if world > 1:
            # RCCL over xGMI on torch's stream; the all-pairs call below is queued
            # on the same stream, so no host sync in between (events time it)
            ev[0].record()
            hh, nn = gather_sketches(loc_h, loc_n)
            ev[1].record()
        else:
            hh, nn = loc_h, loc_n
        part_ms = 0.0
        if sharded:
            part_ms = allpairs_sharded(hh, nn)
        elif seg:
            ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, r0, r1, d_common.data_ptr(), None, stream)
        if record and seg:
            read_kms((2, 3, 4))
            kms[4][0] += part_ms               # the sharded screen's part (its own library call)
        if nloc and ctx.sketch_wait():
            # a genome needed another threshold round: the sketches were redone.
            # One rank alone cannot redo the gather (the other ranks would hang
            # in it), so at world > 1 the step is flagged and the timing rerun
            # with the synchronous check (below); at world = 1 redo the all-pairs
            redo["n"] += 1
            if world == 1 and seg:
                ctx.allpairs_device(hh.data_ptr(), nn.data_ptr(), N, r0, r1, d_common.data_ptr(), None, stream)
        if record and nloc and args.defer_check:
            read_kms((0, 1))
        if record:
            if world > 1:
                ev[1].synchronize()
            stage["gather"] += ev[0].elapsed_time(ev[1]) / 1e3 if world > 1 else 0.0

    def pipelined(nsteps, record):
        """nsteps steps with the host one step ahead: step i's sketch is queued
        before the host waits for step i-1's all-pairs, and every step's checks
        (sketch threshold status, table-build failures) run while the next
        step's kernels execute.  Same work per step as step()."""
        gev = []

        def check_sketch():
            if nloc and ctx.sketch_wait():
                redo["n"] += 1          # sketches rewritten after their all-pairs: re-time (below)
            if record and nloc:
                read_kms((0,))

        for i in range(nsteps):
            if i > 0:
                check_sketch()
            if nloc:
                ctx.sketch_device_async(codes.data_ptr(), valid.data_ptr(), base_off, padded, nkmers, nloc,
                                        loc_h.data_ptr(), loc_n.data_ptr(), stream)
            if i > 0 and seg:
                ctx.allpairs_wait()
            if world > 1:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                hh, nn = gather_sketches(loc_h, loc_n)
                e1.record()
                gev.append((e0, e1))
            else:
                hh, nn = loc_h, loc_n
            if sharded:
                allpairs_sharded(hh, nn)
            elif seg:
                ctx.allpairs_device_async(hh.data_ptr(), nn.data_ptr(), N, r0, r1, d_common.data_ptr(), None,
                                          stream)
        if nsteps:
            check_sketch()
            if seg:
                ctx.allpairs_wait()
        if record and gev:
            gev[-1][1].synchronize()
            stage["gather"] += sum(a.elapsed_time(b) for a, b in gev) / 1e3

    def timed():
        if args.pipeline:
            pipelined(args.warmup, False)
        else:
            for _ in range(args.warmup):
                step(False)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if args.pipeline:
            pipelined(args.steps, True)
        else:
            for _ in range(args.steps):
                step(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el, float(redo["n"])], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el, redo["n"] = float(t[0].item()), int(t[1].item())
        return el

    elapsed = timed()
    if redo["n"] and (world > 1 or args.pipeline):
        # some rank redid its sketches inside a step: those steps' all-pairs
        # used stale sketches, so time again with the synchronous check
        print("bench: a sketch needed another threshold round; re-timing with the synchronous check",
              file=sys.stderr)
        args.defer_check = 0
        args.pipeline = 0
        redo["n"] = 0
        for w in kms:
            kms[w] = [0.0, 0]
        stage["gather"] = 0.0
        elapsed = timed()

    # the timed (possibly pipelined) steps' outputs, checked below (oracle
    # sample by default; --verify: the whole job recomputed on this GPU)
    snap = (loc_h.clone(), loc_n.clone(), d_common.clone()) if (args.verify or args.check) else None

    # ---- the other kernels' times: PROFILE_STEPS extra steps, every kernel
    # bracketed by events (not part of the timed region)
    keep = (list(kms[0]), dict(stage))
    ctx.set_timing(True)
    for w in (1, 2, 3, 4):
        kms[w] = [0.0, 0]
    for _ in range(PROFILE_STEPS):
        step(True)
    torch.cuda.synchronize()
    kms[0], stage = keep
    ctx.set_timing(True, kernels=(0,))
    screen = ctx.screen_stats()

    K = args.steps
    # stage split per step from the kernels' HIP events (the host cannot see
    # it: sketch, gather and all-pairs are queued back to back): sketch = hash
    # kernel (timed steps) + finalize (extra steps); dist = the rest
    stage["sketch"] = K * (kms[0][0] / max(kms[0][1], 1) + kms[1][0] / max(kms[1][1], 1)) / 1e3
    stage["dist"] = max(elapsed - stage["sketch"] - stage["gather"], 0.0)
    if world > 1:
        st = torch.tensor([stage["sketch"], stage["gather"], stage["dist"]], dtype=torch.float64, device=dev)
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        stage = dict(zip(["sketch", "gather", "dist"], st.tolist()))
    ms_step = elapsed / K * 1e3
    pairs = N * (N - 1) / 2
    value = pairs / (elapsed / K)

    # ---- roofline of the dominant kernel (sketch hash), this rank's launches
    sk_ms, sk_n = kms[0]
    avg_launch_s = (sk_ms / max(sk_n, 1)) / 1e3
    alg_bytes = nloc * P * 3 / 8                     # 2-bit codes + 1 validity bit per base
    achieved = alg_bytes / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    # HBM bytes per launch from the committed PMC passes of this build and this
    # launch size (tools/profile_round.sh), else null with the reason
    tj, traffic_src, traffic_note = find_profile(SKETCH_TRAFFIC_NAME, lambda d: d.get("genomes_per_launch") == nloc)
    traffic = tj.get("hbm_bytes_per_launch") if tj else None
    kmers_per_s = nloc * (L - 20) / avg_launch_s if avg_launch_s > 0 else 0.0
    window_ends = nloc * P                           # every padded position is a window end the kernel visits
    valu = {"kmers_per_s": kmers_per_s}
    if os.path.exists(SKETCH_PHASES):
        ph = json.load(open(SKETCH_PHASES))
        valu.update({"kernel": ph["kernel"], "valu_per_kmer_hot_loop": ph["valu_per_kmer"],
                     "valu_per_kmer_by_phase": {k: v["valu_per_kmer"] for k, v in ph["phases"].items()},
                     "isa_source": os.path.relpath(SKETCH_PHASES, ROOT) + " (tools/isa_phases.py)"})
    pmc_doc, pmc_src, pmc_note = find_profile(SKETCH_PMC_NAME)
    pmc_sk = pmc_block(pmc_doc, pmc_src) or {"note": pmc_note}
    if os.path.exists(SKETCH_PRICED) and valu.get("valu_per_kmer_hot_loop") and avg_launch_s > 0:
        # One binding resource: VALU issue of the hot loop's instruction stream.
        # achieved = the hot loop's wave64 VALU instructions per launch / this
        # launch's live time; peak = the same stream at its measured prices
        # (the priced model's mean ns per instruction, every SIMD busy)
        pr = json.load(open(SKETCH_PRICED))
        wi = valu["valu_per_kmer_hot_loop"] * window_ends / 64
        ach = wi / avg_launch_s
        ns = pr["valu_ns_per_instruction_avg"]
        peak = N_SIMD / (ns * 1e-9)
        valu.update({"bound": "valu_issue", "achieved": ach, "peak": peak, "unit": "wave64 VALU instructions/s",
                     "frac": ach / peak,
                     "priced_ns_per_wave_inst_per_simd": ns,
                     "priced_valu_per_kmer": pr["valu_per_kmer"],
                     "peak_source": os.path.relpath(SKETCH_PRICED, ROOT) + " (tools/sketch_priced.py)",
                     "frac_of_2cyc_issue_peak": ach / VALU_PEAK_WAVE_INST,
                     "note": "binding resource: VALU issue. peak = the hot loop's own instructions at their measured "
                             "prices (tools/valu_microbench.hip, 8 waves/SIMD); the priced model predicts "
                             "%.2f ms for the configs[1] launch against %.2f ms measured on the same box; LDS reads "
                             "and SALU add no measurable time to a VALU-bound stream" %
                             (pr["predicted_ms"], pr["measured_hash_ms"])})
        if abs(pr["valu_per_kmer"] - valu["valu_per_kmer_hot_loop"]) > 0.01:         # (the phases file rounds to 3 places)
            valu["note"] += "; the priced mix (%.3f VALU/k-mer) is not this build's (%.3f)" % (
                pr["valu_per_kmer"], valu["valu_per_kmer_hot_loop"])

    # ---- output segment D2H (PCIe-inclusive leg; not part of `value`)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_seg = d_common.cpu()
    d2h_ms = (time.perf_counter() - t0) * 1e3

    verified = None
    if args.verify:
        # the sharded result against this GPU doing the whole job alone
        tot = tile + N * P
        codes_a = torch.zeros(tot // 16, dtype=torch.int32, device=dev)
        valid_a = torch.zeros(tot // 32, dtype=torch.int32, device=dev)
        ctx.synth_device(args.seed, 0, N, args.family_size, L, codes_a.data_ptr(), valid_a.data_ptr(), stream)
        full_h = torch.full((N, s), -1, dtype=torch.int64, device=dev)
        full_n = torch.zeros(N, dtype=torch.int32, device=dev)
        ctx.sketch_device(codes_a.data_ptr(), valid_a.data_ptr(), np.array([tile + i * P for i in range(N)], np.uint64),
                          np.full(N, P, np.uint64), np.full(N, L - 20, np.uint64), N,
                          full_h.data_ptr(), full_n.data_ptr(), stream)
        full_c = torch.zeros(max(N * (N - 1) // 2, 1), dtype=torch.int16, device=dev)
        ctx.allpairs_device(full_h.data_ptr(), full_n.data_ptr(), N, 0, N, full_c.data_ptr(), None, stream)
        torch.cuda.synchronize()
        a = cond_start(r0, N)
        ok = True
        for lh, ln, dc in ((loc_h, loc_n, d_common), snap):     # after the extra steps; after the timed ones
            hh, nn = (gather_sketches(lh, ln) if world > 1 else (lh, ln))
            ok = ok and (torch.equal(hh[:N], full_h) and torch.equal(nn[:N], full_n) and
                         torch.equal(dc[:seg], full_c[a:a + seg]))
        if world > 1:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = bool(flag.item())
        verified = bool(ok)
        del codes_a, valid_a, full_h, full_n, full_c

    checked = None
    if args.check:
        checked = check_against_oracle(args, snap[0], snap[1], snap[2], g0, nloc, N, r0, r1, world, gather_sketches)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        # `mash dist -p <all host cores>` (d_cluster.py:570): every CPU this
        # job may use (affinity, cgroup quota, OMP_NUM_THREADS)
        threads, share = host_cpu_share()
        cpu = cpu_baseline(args, threads, share)

    if rank == 0:
        out = {
            "metric": "genome pairs/sec (mash dist, k=21 s=1000) + sketch GB/s, at 1/2/4/8 GPUs",
            "value": value,
            "unit": "genome pairs/s",
            "value_kind": "end to end: N(N-1)/2 / whole step (sketch + sketch exchange + all-pairs), inputs in HBM",
            "dist_pairs_per_s": pairs / (stage["dist"] / K) if stage["dist"] else None,
            "dist_pairs_per_s_kind": "the metric's quantity (SURVEY.md 8(d)): N(N-1)/2 / all-pairs stage time "
                                     "per step, sketches resident",
            "n_gpus": world,
            "ranks_seen": dist.get_world_size() if world > 1 else 1,
            "backend": (backend if world > 1 else None),
            "rccl_version": rccl_version(torch) if world > 1 and backend == "nccl" else None,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (on-device splitmix64 genome families, 2-bit packed; see DESIGN.md)",
            "config": {
                "workload": "%d synthetic %d bp genomes, k=21, s=%d (%s); step = %s"
                            % (N, L, s, config_name(N, L, s),
                               "sketch shard + RCCL all-gather of sketches + all-pairs row shard" if world > 1
                               else "sketch + all-pairs (one GPU: no all-gather)"),
                "genomes": N, "genome_bp": L, "k": 21, "sketch": s, "family_size": args.family_size,
                "parallelism": "sketch: genome shards; all-pairs: balanced row shards; RCCL all-gather",
                "host_loop": ("pipelined: step i+1 queued before step i's checks" if args.pipeline
                              else "one step at a time") + (", deferred sketch check" if args.defer_check else ""),
            },
            "stages": {
                "sketch_ms_per_step": stage["sketch"] / K * 1e3,
                "allgather_ms_per_step": stage["gather"] / K * 1e3,
                "dist_ms_per_step": stage["dist"] / K * 1e3,
                "sketch_GBps": N * L / (stage["sketch"] / K) / 1e9 if stage["sketch"] else None,
                "sketch_packed_GBps": N * P * 3 / 8 / (stage["sketch"] / K) / 1e9 if stage["sketch"] else None,
                "dist_pairs_per_s": pairs / (stage["dist"] / K) if stage["dist"] else None,
                "output_d2h_ms_rank0": d2h_ms,
                "output_bytes_rank0": int(host_seg.numel() * 2),
            },
            "kernels_rank0": {
                "note": "HIP events on the launch stream: sketch_hash over the timed steps; the "
                        "others over %d extra steps after them" % PROFILE_STEPS,
                "sketch_hash_ms_avg": sk_ms / max(sk_n, 1),
                "sketch_finalize_ms_avg": kms[1][0] / max(kms[1][1], 1),
                "allpairs_ms_avg": kms[2][0] / max(kms[2][1], 1),
                "cuckoo_build_ms_avg": kms[3][0] / max(kms[3][1], 1),
                "screen_ms_avg": kms[4][0] / max(kms[4][1], 1),
                "launches": {"sketch_hash": sk_n, "finalize": kms[1][1], "allpairs": kms[2][1],
                             "build": kms[3][1], "screen": kms[4][1]},
            },
            "roofline": {
                "kernel": valu.get("kernel", "k_sketch_hash21"),
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_source": traffic_src or traffic_note,
                "note": "algorithmic bytes = 0.375 B/base (2-bit code + validity bit) x bases per "
                        "launch; HBM is not the limit: the kernel is VALU-issue bound (Murmur3, 63 "
                        "VALU instructions per k-mer in the hot loop), see valu_model",
                "valu_model": valu,
                "pmc": pmc_sk,
            },
            "dist_kernel": {
                "kernel": "k_allpairs_q (s <= 2048) / k_allpairs_band",
                "screen": dict(screen, sharded_by_hash_range=sharded,
                               note="shared-hash screen (screen.hip): the kernel runs only on the (row "
                                    "tile, column) cells whose genomes share a hash; auto from 4096 genomes; "
                                    "with several ranks sharded by hash range (each rank groups one part, "
                                    "the marks exchanged; screen_ms = its part + its rows' finish)"),
                "bound": "VALU + LDS (random slot reads); integer set intersection, no MFMA",
                "ms_per_launch": kms[2][0] / max(kms[2][1], 1),
                "pairs_per_launch": segment_size(N, r0, r1),
                "pairs_per_s_per_gpu": (segment_size(N, r0, r1) / (kms[2][0] / max(kms[2][1], 1) / 1e3)
                                        if kms[2][0] else None),
                "roofline": dist_roofline(N, args.sketch, args.family_size, bool(screen.get("used")),
                                          segment_size(N, r0, r1), kms[2][0] / max(kms[2][1], 1)),
                "screened_stage": ({"note": "screened path (DESIGN.md 4.6): the sort/mark/list passes, the "
                                            "no-shared-hash fill and the LIST kernel on the marked (row tile, column) "
                                            "cells; the roofline above is the LIST kernel's",
                                    "screen_ms_avg": kms[4][0] / max(kms[4][1], 1),
                                    "sort_bytes_per_launch_est": 4 * 16 * screen.get("entries", 0),
                                    "marked_cells": screen.get("marked"), "pair_checks": screen.get("checks")}
                                   if screen.get("used") else None),
            },
            "cpu_baseline": cpu,
        }
        if checked is not None:
            out["verified"] = checked["verified"]
            out["verification"] = dict(checked, how="timed steps' outputs vs the C oracle: sampled genomes "
                                       "re-sketched on the host; random pairs + one whole row re-merged")
        if verified is not None:
            out["verified_against_single_gpu"] = verified
        print(json.dumps(out))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def rccl_version(torch):
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception as e:
        return "unknown (%s)" % e


if __name__ == "__main__":
    sys.exit(main() or 0)
