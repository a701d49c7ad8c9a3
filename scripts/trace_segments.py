"""Split a rocprofv3 kernel trace into launch bursts (gaps > 1 ms) and break down the last burst
with at least `min_kernels` kernels.  Usage: trace_segments.py trace.csv [min_kernels] [top]"""
import collections
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    mk = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    segs = [[rows[0]]]
    for a, b in zip(rows, rows[1:]):
        if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 1_000_000:
            segs.append([])
        segs[-1].append(b)
    seg = [s for s in segs if len(s) >= mk][-1]
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
    print(f"{len(seg)} kernels, span {span:.1f} us, busy {busy:.1f} us")
    tot = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = r["Kernel_Name"][:64] + " g=" + r["Grid_Size_X"] + "x" + r["Grid_Size_Y"] + "x" + r["Grid_Size_Z"]
        tot[k][0] += 1
        tot[k][1] += d
    for k, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{k:100s} {c:5d} {d / 1e3:9.1f} us")


if __name__ == "__main__":
    main()
