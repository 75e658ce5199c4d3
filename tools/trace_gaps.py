"""Timeline of the last kernels in a rocprofv3 kernel-trace CSV: each
dispatch's duration and the idle gap before it (not part of the product).
    python tools/trace_gaps.py <kernel_trace.csv> [last_n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-n:]:
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (a - prev) / 1e3 if prev is not None else 0.0
    print("%9.1f us gap %8.1f us  %s" % (gap, (b - a) / 1e3, r["Kernel_Name"][:90]))
    prev = b
