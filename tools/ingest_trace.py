"""Kernel + copy timeline of the overlapped FASTA ingest (not part of the
product).  Reads a rocprofv3 output directory made with --kernel-trace
--memory-copy-trace around tools/ingest_bench.py and prints, per
drephip_sketch_files batch, when its host-to-device copies and its sketch
kernels ran, plus the GPU-idle time between batches (the host producer
packing the next batch).

usage: python tools/ingest_trace.py <rocprof dir> [gap_ms] > profiles/<round>_ingest_trace.json
"""
import csv
import glob
import json
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        out.extend(csv.DictReader(open(f)))
    return out


def main():
    d = sys.argv[1]
    kern = rows(d + "/**/*kernel_trace.csv")
    copy = rows(d + "/**/*memory_copy_trace.csv")
    ev = []
    for r in kern:
        name = r["Kernel_Name"]
        kind = ("hash" if "k_sketch_hash21" in name else "finalize" if "finalize" in name else
                "tables" if "k_sketch_tables" in name else "reset" if "reset" in name else "other")
        ev.append({"t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"]), "kind": kind, "bytes": 0})
    for r in copy:
        direction = r.get("Direction") or r.get("Operation") or ""
        size = int(r.get("Size") or r.get("Bytes") or 0)
        kind = "h2d" if "HOST_TO_DEVICE" in direction.upper() or "H2D" in direction.upper() else "d2h" \
            if "DEVICE_TO_HOST" in direction.upper() or "D2H" in direction.upper() else "copy"
        ev.append({"t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"]), "kind": kind, "bytes": size})
    ev.sort(key=lambda e: e["t0"])
    if not ev:
        print(json.dumps({"error": "no events", "dir": d}))
        return
    # batches: runs of GPU events separated by idle gaps longer than GAP_MS
    # (the producer thread reading and packing the next batch); the trace has
    # no copy sizes, so bytes come from the durations only
    GAP_MS = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    batches, cur, last = [], None, None
    for e in ev:
        if cur is None or (e["t0"] - last) / 1e6 > GAP_MS:
            cur = {"h2d_n": 0, "h2d_ms": 0.0, "hash_ms": 0.0, "finalize_ms": 0.0, "other_ms": 0.0,
                   "t0": e["t0"], "t1": e["t1"]}
            batches.append(cur)
        cur["t1"] = max(cur["t1"], e["t1"])
        last = cur["t1"]
        if e["kind"] == "h2d":
            cur["h2d_n"] += 1
            cur["h2d_ms"] += (e["t1"] - e["t0"]) / 1e6
        elif e["kind"] in ("hash", "finalize"):
            cur[e["kind"] + "_ms"] += (e["t1"] - e["t0"]) / 1e6
        else:
            cur["other_ms"] += (e["t1"] - e["t0"]) / 1e6
    t_first = ev[0]["t0"]
    out = {"source": d, "events": len(ev), "batches": []}
    prev_end = None
    for b in batches:
        out["batches"].append({"start_ms": (b["t0"] - t_first) / 1e6, "end_ms": (b["t1"] - t_first) / 1e6,
                               "gpu_idle_before_ms": None if prev_end is None else (b["t0"] - prev_end) / 1e6,
                               "h2d_copies": b["h2d_n"], "h2d_ms": b["h2d_ms"], "hash_ms": b["hash_ms"],
                               "finalize_ms": b["finalize_ms"], "other_ms": b["other_ms"]})
        prev_end = b["t1"]
    busy = sum((e["t1"] - e["t0"]) for e in ev) / 1e6
    out["span_ms"] = (max(e["t1"] for e in ev) - t_first) / 1e6
    out["gpu_busy_ms"] = busy
    out["note"] = ("each batch's copies + kernels run while the producer thread packs the next batch; "
                   "gpu_idle_before_ms is the host-bound part (read + decompress + pack) not hidden")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
