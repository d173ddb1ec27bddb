"""Per-kernel duration, effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and cycles per
instruction from a rocprofv3 --pmc GRBM_GUI_ACTIVE ... counter_collection.csv.
Usage: python pmc_clock.py CSV [instructions_per_wave]"""
import collections
import csv
import sys


def main():
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(sys.argv[1])):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"][:48])
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    ipw = float(sys.argv[2]) if len(sys.argv) > 2 else 0
    agg = collections.defaultdict(list)
    for k in sorted(d):
        s, e = meta[k]
        ga = d[k]["GRBM_GUI_ACTIVE"] / 8
        agg[k[1]].append(((e - s) / 1e6, ga / (e - s), ga))
    for n, v in agg.items():
        v = v[2:] if len(v) > 3 else v  # drop the warm-up launches
        ms = sum(x[0] for x in v) / len(v)
        ghz = sum(x[1] for x in v) / len(v)
        cyc = sum(x[2] for x in v) / len(v)
        extra = "  %.2f cycles/instr" % (cyc / ipw) if ipw else ""
        print("%-48s %.4f ms  %.3f GHz  %.0f cycles%s" % (n, ms, ghz, cyc, extra))


if __name__ == "__main__":
    main()
