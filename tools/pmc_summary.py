"""Sum rocprofv3 PMC counter passes per kernel into one JSON (not part of the
product).  usage: python tools/pmc_summary.py <kernel substring> <csv>... > out.json"""
import collections
import csv
import json
import sys


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
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
