"""Median / mean per kernel over a rocprofv3 kernel trace, for every p_* directory of an A/B run."""
import csv
import glob
import os
import statistics
import sys

for p in sorted(glob.glob(os.path.join(sys.argv[1], "p_*"))):
    f = glob.glob(os.path.join(p, "*kernel_trace.csv"))[0]
    d = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if any(x in k for x in ("solve", "apply", "colprog_K1024_n76")):
            d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    out = []
    for k, v in sorted(d.items()):
        out.append("%s med %.1f mean %.1f" % (k.replace("void rq::", "")[:24], statistics.median(v), statistics.mean(v)))
    print(os.path.basename(p), " | ".join(out))
