"""Per-setting kernel averages (us) of an A/B directory written by sx_ab.sh / solve_ab.sh, beside the
decode_ms lines of its ab.log."""
import csv
import glob
import os
import sys

d = sys.argv[1]
print("".join(l for l in open(os.path.join(d, "ab.log")) if l.startswith(("==", "decode_ms", "solved"))))
for p in sorted(glob.glob(os.path.join(d, "p_*"))):
    f = glob.glob(os.path.join(p, "*kernel_stats.csv"))[0]
    row = []
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("solve", "apply", "colprog_K1024_n76")):
            row.append("%s %.1f" % (r["Name"].replace("void rq::", "")[:28], float(r["AverageNs"]) / 1000))
    print(os.path.basename(p), " | ".join(row))
