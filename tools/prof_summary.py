"""Summarise rocprofv3 CSV output for profiles/: per (kernel, grid) launch shape the count and mean
duration from *_kernel_trace.csv, and per-dispatch HBM bytes from *_counter_collection.csv
(FETCH_SIZE / WRITE_SIZE are in KiB)."""
import csv, json, sys
from collections import defaultdict


def trace_summary(path):
    g = defaultdict(list)
    for r in csv.DictReader(open(path)):
        g[(r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) if "Grid_Size_X" in r else r.get("Grid_Size"))].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = []
    for (k, grid), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        out.append({"kernel": k, "grid_threads": grid, "calls": len(d), "mean_us": round(sum(d) / len(d) / 1e3, 2),
                    "min_us": round(min(d) / 1e3, 2), "max_us": round(max(d) / 1e3, 2)})
    return out


def counter_summary(path):
    g = defaultdict(list)
    for r in csv.DictReader(open(path)):
        g[(r["Kernel_Name"], r["Grid_Size"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return [{"kernel": k, "grid_threads": int(grid), "counter": c, "dispatches": len(v),
             "mean_bytes": round(sum(v) / len(v) * 1024)} for (k, grid, c), v in g.items()]


if __name__ == "__main__":
    res = {"trace": trace_summary(sys.argv[1]), "counters": []}
    for p in sys.argv[2:]:
        res["counters"] += counter_summary(p)
    print(json.dumps(res, indent=1))
