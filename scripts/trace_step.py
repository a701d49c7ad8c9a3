"""Summarise the last decode steps of a rocprofv3 kernel trace: per-kernel device time, launches and
the idle gaps between consecutive kernels.  Usage: trace_step.py <kernel_trace.csv> [n_last_dispatches]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n_last:]
t0 = int(rows[0]["Start_Timestamp"])
t1 = int(rows[-1]["End_Timestamp"])
busy = collections.defaultdict(float)
cnt = collections.Counter()
gap = 0.0
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:70]
    busy[name] += (e - s) / 1e3
    cnt[name] += 1
    if prev_end is not None and s > prev_end:
        gap += (s - prev_end) / 1e3
    prev_end = max(prev_end or 0, e)
span = (t1 - t0) / 1e3
print(f"dispatches {len(rows)}  span {span:.1f} us  busy {sum(busy.values()):.1f} us  idle gaps {gap:.1f} us")
for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
    print(f"  {k:70s} n={cnt[k]:5d} total={v:9.1f} us avg={v / cnt[k]:7.2f} us")
