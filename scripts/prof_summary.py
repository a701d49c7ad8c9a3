"""Summarize a rocprofv3 --kernel-trace CSV: top kernels by total time, and per-launch-shape
breakdown for kernels matching a substring.  Usage: prof_summary.py trace.csv [substr ...]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    tot = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        t = tot[r["Kernel_Name"]]
        t[0] += 1
        t[1] += d
    all_ns = sum(v[1] for v in tot.values())
    print(f"total kernel time {all_ns / 1e6:.3f} ms over {sum(v[0] for v in tot.values())} launches")
    for name, (n, ns) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:18]:
        print(f"{name[:72]:72s} {n:6d} {ns / 1e6:9.3f} ms {ns / n / 1e3:9.2f} us {100 * ns / all_ns:5.1f}%")
    for sub in sys.argv[2:]:
        g = collections.defaultdict(list)
        for r in rows:
            if sub in r["Kernel_Name"]:
                g[(r["Kernel_Name"][:40], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])].append(
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
            print(" ", k, len(v), f"{sum(v) / len(v) / 1e3:.1f} us avg")


if __name__ == "__main__":
    main()
