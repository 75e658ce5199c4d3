"""Sum rocprofv3 PMC counter passes per kernel into one JSON (not part of the
product).

usage: python tools/pmc_summary.py <kernel substring> <csv>... [--window-ends N] [--kernel-ms T] > out.json

Derived quantities (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units"):
  * SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles; busy and
    wait fractions below are ratios of like units;
  * GRBM_GUI_ACTIVE rides along in every pass and rocprofv3 sums it over the 8
    XCDs: kernel cycles per dispatch = sum / passes / 8 / dispatches;
  * valu_issue_frac_2cyc = SQ_INSTS_VALU x 2 / (1024 SIMDs x kernel cycles):
    VALU issue against the guide's peak of one wave64 instruction per 2 cycles
    per SIMD (SIMD-32).  Integer 3-operand and 64-bit instructions measure
    ~2.6 cycles and the simple ones ~1.45 (profiles/r01_valu_microbench.json),
    so a mix-priced bound sits between this and 1.3x it;
  * valu_active_quad_frac = SQ_ACTIVE_INST_VALU (quad-cycles) x 4 / (1024 SIMDs
    x kernel cycles): the counter's own unit (it equals SQ_INSTS_VALU, one
    quad-cycle per instruction), i.e. the share at a 4-cycle issue;
  * lds_busy_frac = SQ_LDS_IDX_ACTIVE (LDS-array cycles per CU) / (256 CUs x
    kernel cycles); lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT /
    SQ_LDS_IDX_ACTIVE (the extra cycles conflicts cost);
  * --window-ends: positions the sketch kernel visits per dispatch, for
    valu_insts_per_window_end = wave64 VALU instructions x 64 / window ends;
  * --kernel-ms: average dispatch time (rocprofv3 --stats), for the effective
    clock = kernel cycles / time.
"""
import argparse
import collections
import csv
import json

N_CU, N_SIMD = 256, 1024          # MI355X


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("files", nargs="+")
    ap.add_argument("--window-ends", type=float, default=None)
    ap.add_argument("--kernel-ms", type=float, default=None)
    a = ap.parse_args()
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    passes_with_grbm = 0
    name = None
    for f in a.files:
        seen_grbm = False
        for r in csv.DictReader(open(f)):
            if a.key in r["Kernel_Name"]:
                name = r["Kernel_Name"]
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
                seen_grbm |= r["Counter_Name"] == "GRBM_GUI_ACTIVE"
        passes_with_grbm += seen_grbm
    out = {"kernel": name, "counters": dict(agg), "dispatches": {k: len(v) for k, v in disp.items()}}
    c = agg
    d = out.setdefault("derived", {})
    if c.get("SQ_WAVE_CYCLES"):
        d["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
        d["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        d["active_inst_any_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
    ndisp = max(len(disp.get("SQ_INSTS_VALU", ())), 1)
    if c.get("SQ_WAVES"):
        d["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
    if c.get("SQ_INSTS_VALU") and a.window_ends:
        d["valu_insts_per_window_end"] = c["SQ_INSTS_VALU"] / ndisp * 64 / a.window_ends
    if c.get("GRBM_GUI_ACTIVE"):
        # every (pass, dispatch) adds one GRBM reading summed over the 8 XCDs
        cyc = c["GRBM_GUI_ACTIVE"] / 8 / max(len(disp["GRBM_GUI_ACTIVE"]), 1)        # per dispatch
        d["kernel_cycles_per_dispatch"] = cyc
        if a.kernel_ms:
            d["effective_clock_ghz"] = cyc / (a.kernel_ms * 1e-3) / 1e9
        if c.get("SQ_INSTS_VALU"):
            d["valu_issue_frac_2cyc"] = c["SQ_INSTS_VALU"] / ndisp * 2 / (N_SIMD * cyc)
        vd = max(len(disp.get("SQ_ACTIVE_INST_VALU", ())), 1)
        if c.get("SQ_ACTIVE_INST_VALU"):
            d["valu_active_quad_frac"] = c["SQ_ACTIVE_INST_VALU"] / vd * 4 / (N_SIMD * cyc)
        ld = max(len(disp.get("SQ_LDS_IDX_ACTIVE", ())), 1)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_busy_frac"] = c["SQ_LDS_IDX_ACTIVE"] / ld / (N_CU * cyc)
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from drep_amd import _lib
    out["build_id"] = _lib.build_id()          # the library the profiled command loaded
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
