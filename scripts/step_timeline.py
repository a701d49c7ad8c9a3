"""One decode step of a rocprofv3 --kernel-trace CSV as a timeline: every kernel between the last two
launches of the step's first kernel (default k_embed_sum), with its duration and the idle gap before it,
then per-kernel totals over that step.  Usage: step_timeline.py trace.csv [first_kernel_substr]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "k_embed_sum"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # one queue: the busiest one (a single-replica run has one decode stream)
    q = collections.Counter(r.get("Queue_Id", "0") for r in rows)
    qid = q.most_common(1)[0][0]
    rows = [r for r in rows if r.get("Queue_Id", "0") == qid]
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    if len(starts) < 3:
        print("fewer than 3 steps found")
        return
    a, b = starts[-3], starts[-2]
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    t_end = int(rows[b]["Start_Timestamp"])
    busy = 0
    prev_end = t0
    per = collections.defaultdict(lambda: [0, 0, 0])
    print(f"step: {len(step)} kernels, {(t_end - t0) / 1e3:.1f} us start to next start")
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d, gap = e - s, s - prev_end
        busy += d
        prev_end = max(prev_end, e)
        name = r["Kernel_Name"].split("(")[0][:60]
        p = per[name]
        p[0] += 1
        p[1] += d
        p[2] += max(gap, 0)
        if "-v" in sys.argv:
            print(f"  {(s - t0) / 1e3:8.1f} {d / 1e3:7.2f} gap {gap / 1e3:6.2f}  {name} grid {r['Grid_Size_X']}")
    print(f"busy {busy / 1e3:.1f} us, idle {(t_end - t0 - busy) / 1e3:.1f} us")
    for name, (n, d, g) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {name:60s} {n:4d} x {d / n / 1e3:6.2f} us = {d / 1e3:7.1f} us, gaps before {g / 1e3:6.1f} us")


if __name__ == "__main__":
    main()
