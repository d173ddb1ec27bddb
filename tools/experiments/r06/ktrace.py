"""Per-kernel durations and the gaps before them from a rocprofv3 kernel trace (the last N dispatches)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
prev = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0
    print("%-40s %8.1f us  gap %6.1f" % (r["Kernel_Name"].replace("void rq::", "")[:40], (e - s) / 1000, gap))
    prev = e
