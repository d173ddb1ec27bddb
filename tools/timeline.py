"""One bench step's GPU timeline from a rocprofv3 kernel trace (+ memory-copy trace): each kernel and
copy with its duration and the idle gap before it.  usage: python tools/timeline.py KERNEL_TRACE.csv
[MEMCPY_TRACE.csv] [step_marker_kernel]"""
import csv
import sys


def main():
    ev = []
    for r in csv.DictReader(open(sys.argv[1])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]))
    if len(sys.argv) > 2 and sys.argv[2].endswith(".csv"):
        for r in csv.DictReader(open(sys.argv[2])):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
    ev.sort()
    marker = sys.argv[-1] if not sys.argv[-1].endswith(".csv") else "rq_colprog_K1024_n76"
    idx = [i for i, e in enumerate(ev) if e[2].startswith(marker)]
    if len(idx) < 3:
        print("marker not found"); return
    a, b = idx[-3], idx[-2]  # one full step near the end
    prev_end = ev[a - 1][1]
    tot_gap = 0
    for s, e, n in ev[a:b]:
        gap = max(0, s - prev_end)
        tot_gap += gap
        print("%-42s %9.1f us   gap %7.1f us" % (n, (e - s) / 1e3, gap / 1e3))
        prev_end = max(prev_end, e)
    print("step %.1f us, idle gaps %.1f us" % ((ev[b][0] - ev[a][0]) / 1e3, tot_gap / 1e3))


if __name__ == "__main__":
    main()
