"""Sum rocprofv3 PMC counter passes per kernel into one JSON (not part of the
product).  usage: python tools/pmc_summary.py <kernel substring> <csv>... > out.json"""
import collections
import csv
import json
import sys

N_CU, N_SIMD = 256, 1024          # MI355X

def main():
    key, files = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    name = None
    for f in files:
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                name = r["Kernel_Name"]
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    out = {"kernel": name, "counters": dict(agg), "dispatches": {k: len(v) for k, v in disp.items()}}
    c = agg
    if c.get("SQ_WAVE_CYCLES"):
        out["derived"] = {
            "wait_any_frac": c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"],
            "wait_inst_any_frac": c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"],
            "active_inst_any_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"],
        }
    if c.get("SQ_LDS_IDX_ACTIVE"):
        out.setdefault("derived", {})["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
    if c.get("SQ_WAVES"):
        out.setdefault("derived", {})["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
    # GRBM_GUI_ACTIVE rides along in every pass and rocprofv3 sums it over the 8
    # XCDs: kernel cycles = sum / passes / 8.  A wave64 VALU instruction holds a
    # SIMD for 4 cycles (SQ_ACTIVE_INST_VALU counts 1 per instruction here);
    # SQ_LDS_IDX_ACTIVE counts LDS-array cycles per CU.
    npass = len(disp.get("GRBM_GUI_ACTIVE", ())) or 1
    npass = max(1, sum(1 for f in files if any(key in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"
                                               for r in csv.DictReader(open(f)))))
    if c.get("GRBM_GUI_ACTIVE"):
        cyc = c["GRBM_GUI_ACTIVE"] / npass / 8
        d = out.setdefault("derived", {})
        d["kernel_cycles"] = cyc
        if c.get("SQ_ACTIVE_INST_VALU"):
            d["valu_busy_frac"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (N_SIMD * cyc)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_busy_frac"] = c["SQ_LDS_IDX_ACTIVE"] / (N_CU * cyc)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
