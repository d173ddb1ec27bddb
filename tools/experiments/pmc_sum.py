"""Per-launch sums of rocprofv3 --pmc counter CSVs under DIR (run.sh's pmc step)."""
import csv
import glob
import sys

for f in sorted(glob.glob(sys.argv[1] + '/p*/**/*counter_collection.csv', recursive=True)):
    rows = list(csv.DictReader(open(f)))
    agg, disp = {}, set()
    for r in rows:
        agg[r['Counter_Name']] = agg.get(r['Counter_Name'], 0) + float(r['Counter_Value'])
        disp.add(r['Dispatch_Id'])
    name = rows[0]['Kernel_Name'][:48] if rows else ''
    print(f, len(disp), name, {k: round(v / max(1, len(disp))) for k, v in sorted(agg.items())})
