"""Per-AR-step device busy time vs span from a rocprofv3 kernel trace: steps are delimited by
k_greedy_step dispatches.  Usage: step_gaps.py <kernel_trace.csv>"""
import csv
import sys
import collections

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "k_greedy_step" in r["Kernel_Name"]]
spans, busys, per = [], [], collections.defaultdict(float)
for a, b in zip(marks[5:], marks[6:]):
    seg = rows[a + 1:b + 1]
    s0, s1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    spans.append((s1 - s0) / 1e3)
    busys.append(busy / 1e3)
    for r in seg:
        per[r["Kernel_Name"].split("(")[0][:60]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
n = len(spans)
print(f"steps {n}  span/step {sum(spans)/n:.1f} us  busy/step {sum(busys)/n:.1f} us  kernels/step {(marks[-1]-marks[5])/n:.1f}")
for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:16]:
    print(f"  {k:60s} {v/n:8.1f} us/step")
