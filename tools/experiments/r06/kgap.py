"""Median gap (us) before each kernel kind in a rocprofv3 kernel trace, for every p_* directory of an A/B run."""
import csv
import glob
import os
import statistics
import sys

for p in sorted(glob.glob(os.path.join(sys.argv[1], "p_*"))):
    rows = list(csv.DictReader(open(glob.glob(os.path.join(p, "*kernel_trace.csv"))[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gaps, prev, pk = {}, None, None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = r["Kernel_Name"].replace("void rq::", "")[:20]
        if prev is not None and pk is not None:
            gaps.setdefault(pk + " -> " + k, []).append((s - prev) / 1000)
        prev, pk = e, k
    print(os.path.basename(p), " | ".join("%s %.1f (%d)" % (k, statistics.median(v), len(v))
                                          for k, v in sorted(gaps.items()) if len(v) > 20))
