"""One JSON per all-pairs profiling case of tools/profile_allpairs.sh (not part
of the product): average dispatch time from the kernel trace, and per
dispatch the HBM traffic (FETCH_SIZE / WRITE_SIZE, KB; gfx950 FETCH_SIZE
tallies a coalesced 16-B-per-lane stream at half its bytes -- MI355X_MICROARCH.md
HBM -- so both the raw and the doubled read figure are given: the column loads
here are 8 B per lane, an uncalibrated width), the L2 hit rate, and the SQ
issue/stall fractions (tools/pmc_summary.py's definitions).

usage: python tools/allpairs_traffic_json.py <kernel substring> <dir> <case> N s calls [family_size]

The summary names the workload (N, s, the generator's family size, whether the
profiled dispatches are the screened LIST template or the dense one) and the
library build (drephip_build_id of drep_amd/lib/libdrephip.so, loaded here
without a GPU): bench.py quotes a profile only for its own workload and build.

`calls` = all-pairs calls the profiled command made (bench.py --steps 1
--warmup 0: 4, its three timing steps included; tools/ap_bench.py with
AP_ITERS=1: 1).  A call over a large triangle is several dispatches (grid
limit), so every figure is per CALL = the whole N(N-1)/2 triangle: the sum
over dispatches divided by `calls`.
"""
import collections
import csv
import glob
import json
import os
import sys

N_CU, N_SIMD = 256, 1024


def per_dispatch(files, key):
    """{counter: average per dispatch} over every dispatch of the kernel."""
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    name = None
    for f in files:
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                name = r["Kernel_Name"]
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    return {k: v / max(len(disp[k]), 1) for k, v in agg.items()}, {k: len(v) for k, v in disp.items()}, name


def main():
    key, d, case, N, s = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    ncalls = int(sys.argv[6])
    family = int(sys.argv[7]) if len(sys.argv) > 7 else 100
    stats = glob.glob(os.path.join(d, case + "_trace", "**", "*kernel_stats.csv"), recursive=True)
    avg_ms, ndisp = None, None
    for r in csv.DictReader(open(stats[0])):
        if key in r["Name"]:
            ndisp = int(r["Calls"])
            avg_ms = float(r["AverageNs"]) / 1e6 * ndisp / ncalls        # per call (whole triangle)
    files = sorted(glob.glob(os.path.join(d, case + "_p*", "**", "pmc_counter_collection.csv"), recursive=True))
    cd, nd, name = per_dispatch(files, key)
    # per call: the per-dispatch average times the dispatches of one pass over calls
    passes = len({f for f in files})
    c = {k: v * nd[k] / max(1, passes if k == "GRBM_GUI_ACTIVE" else 1) / ncalls for k, v in cd.items()}
    # GRBM_GUI_ACTIVE rides in every pass (summed over 8 XCDs): its dispatch
    # count above spans all passes, hence the division by the pass count
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from drep_amd import _lib
    variant = "LIST" if name and ("true>" in name or "true," in name) else "dense"
    out = {"case": case, "kernel": name, "kernel_variant": variant, "build_id": _lib.build_id(),
           "workload": {"genomes": N, "sketch": s, "family_size": family, "kernel_variant": variant},
           "genomes": N, "sketch": s, "pairs": N * (N - 1) // 2,
           "calls": ncalls, "dispatches_per_call": (ndisp or 0) / ncalls, "avg_call_ms": avg_ms,
           "counters_per_call": c, "dispatches_per_counter": nd}
    dv = out["derived"] = {}
    if cyc and avg_ms:
        dv["kernel_cycles"] = cyc
        dv["effective_clock_ghz"] = cyc / (avg_ms * 1e-3) / 1e9
    if "FETCH_SIZE" in c:
        raw = c["FETCH_SIZE"] * 1024
        dv["hbm_read_bytes_raw"] = raw
        dv["hbm_read_bytes_x2"] = 2 * raw
    if "WRITE_SIZE" in c:
        dv["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
    alg_read = N * s * 8                                 # every sketch read once
    alg_write = N * (N - 1) // 2 * 2                     # uint16 common per pair
    dv["algorithmic_bytes"] = alg_read + alg_write
    dv["column_stream_bytes_logical"] = (N * (N - 1) // 2) * s * 8 / 4   # every pair's column once per 4-row tile
    if "hbm_read_bytes_raw" in dv and "hbm_write_bytes" in dv and avg_ms:
        for tag in ("raw", "x2"):
            tot = dv["hbm_read_bytes_" + tag] + dv["hbm_write_bytes"]
            dv["hbm_bytes_" + tag] = tot
            dv["hbm_GBps_" + tag] = tot / (avg_ms * 1e-3) / 1e9
        dv["hbm_frac_of_8TBps_x2"] = dv["hbm_GBps_x2"] / 8000.0
        dv["hbm_over_algorithmic_x2"] = dv["hbm_bytes_x2"] / dv["algorithmic_bytes"]
    if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0):
        dv["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        dv["l2_requests"] = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
        if avg_ms:
            dv["l2_req_per_s"] = dv["l2_requests"] / (avg_ms * 1e-3)
    if c.get("SQ_WAVE_CYCLES"):
        dv["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
        dv["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        dv["active_inst_any_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_INSTS_VALU"):
        dv["salu_over_valu"] = c.get("SQ_INSTS_SALU", 0) / c["SQ_INSTS_VALU"]
        dv["valu_wave_insts_per_pair"] = c["SQ_INSTS_VALU"] / max(N * (N - 1) // 2, 1)
        dv["salu_insts_per_pair"] = c.get("SQ_INSTS_SALU", 0) / max(N * (N - 1) // 2, 1)
        if cyc:
            dv["valu_issue_frac_2cyc"] = c["SQ_INSTS_VALU"] * 2 / (N_SIMD * cyc)
    if c.get("SQ_LDS_IDX_ACTIVE") and cyc:
        dv["lds_busy_frac"] = c["SQ_LDS_IDX_ACTIVE"] / (N_CU * cyc)
        dv["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
    if avg_ms:
        dv["pairs_per_s"] = N * (N - 1) / 2 / (avg_ms * 1e-3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
