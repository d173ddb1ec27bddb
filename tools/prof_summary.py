"""Summarise rocprofv3 CSV output for profiles/.

  prof_summary.py trace TRACE_CSV [COUNTER_CSV ...]   per (kernel, grid) count and mean duration,
                                                      plus per-dispatch counter means
  prof_summary.py traffic DIR TAG [KERNEL]            FETCH_SIZE / WRITE_SIZE passes of
                                                      tools/gpu_profile.sh (copied to profiles/TAG_traffic.json;
                                                      KERNEL rq_colprog_K256_n26: TAG_k256_traffic.json)

FETCH_SIZE / WRITE_SIZE are in KiB.  Calibration (MI355X_MICROARCH.md, HBM section): the counters are
exact only for some access widths, so each is divided by its ratio on a same-pattern copy launch of
known byte count (rq_colprog_K10_n10 = load + store of every source row, tools/pmc_workload.py).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def trace_summary(path):
    g = defaultdict(list)
    for r in csv.DictReader(open(path)):
        g[(r["Kernel_Name"], r.get("Grid_Size"))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = []
    for (k, grid), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        out.append({"kernel": k, "grid_threads": grid, "calls": len(d), "mean_us": round(sum(d) / len(d) / 1e3, 2),
                    "min_us": round(min(d) / 1e3, 2), "max_us": round(max(d) / 1e3, 2)})
    return out


def counter_means(path):
    g = defaultdict(list)
    for r in csv.DictReader(open(path)):
        g[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in g.items()}


WORKLOADS = {  # encode launches of tools/pmc_workload.py: kernel -> (K, T, N, blocks)
    "rq_colprog_K1024_n76": (1024, 1200, 1100, 1024),  # the bench metric (config 3)
    "rq_colprog_K256_n26": (256, 1200, 282, 1024),     # BASELINE config 2
}


def traffic(d, tag, enc="rq_colprog_K1024_n76"):
    fetch = counter_means(glob.glob(os.path.join(d, "fetch", "*counter_collection.csv"))[0])
    write = counter_means(glob.glob(os.path.join(d, "write", "*counter_collection.csv"))[0])
    cal_bytes = 65536 * 10 * 1024
    cal = "rq_colprog_K10_n10"
    K, T, N, B = WORKLOADS[enc]
    f_cal, w_cal = fetch[(cal, "FETCH_SIZE")] / cal_bytes, write[(cal, "WRITE_SIZE")] / cal_bytes
    f_enc, w_enc = fetch[(enc, "FETCH_SIZE")] / f_cal, write[(enc, "WRITE_SIZE")] / w_cal
    out = {
        "kernel": enc,
        "workload": {"K": K, "T": T, "N": N, "blocks": B},
        "fetch_bytes": round(f_enc), "write_bytes": round(w_enc), "traffic_bytes": round(f_enc + w_enc),
        "algorithmic_bytes": {"read": B * K * T, "write": B * (N - K) * T},
        "calibration": {"kernel": cal, "bytes_read_and_written": cal_bytes, "fetch_ratio": round(f_cal, 4),
                        "write_ratio": round(w_cal, 4)},
        "raw_kib": {"fetch": fetch[(enc, "FETCH_SIZE")] / 1024, "write": write[(enc, "WRITE_SIZE")] / 1024},
        "source": "tools/gpu_profile.sh: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                  "tools/pmc_workload.py; counters divided by their ratio on the calibration copy",
    }
    out["tag"] = tag
    return out


if __name__ == "__main__":
    if sys.argv[1] == "traffic":
        print(json.dumps(traffic(sys.argv[2], sys.argv[3], *sys.argv[4:5]), indent=1))
    else:
        res = {"trace": trace_summary(sys.argv[2]), "counters": []}
        for p in sys.argv[3:]:
            res["counters"] += [{"kernel": k, "counter": c, "mean_bytes": round(v)} for (k, c), v in counter_means(p).items()]
        print(json.dumps(res, indent=1))
