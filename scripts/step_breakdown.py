"""Per-decode-step kernel breakdown from a rocprofv3 kernel trace of bench.py.
Usage: step_breakdown.py trace.csv [first_step] [n_steps] [marker_grid|-] [marker_name]

Steps are delimited by the device greedy-sampling launches (k_greedy_step*).  The bench runs the
Parler leg first, then Orpheus / Dia; `marker_grid` (Grid_Size_X of the Parler leg's sampling
kernel, e.g. 4608 for 8 prompts x 9 heads x 64 lanes) keeps only that leg's markers.  The step
window is the last n_steps markers before the final `first_step` ones (the profiled roofline pass
at the end of the leg is skipped)."""
import collections
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    grid = sys.argv[4] if len(sys.argv) > 4 and sys.argv[4] != "-" else None
    name = sys.argv[5] if len(sys.argv) > 5 else "k_greedy_step"
    g = [i for i, r in enumerate(rows) if name in r["Kernel_Name"] and (grid is None or r["Grid_Size_X"] == grid)]
    if len(g) < first + n:
        print(f"only {len(g)} step markers")
        n = len(g) - first - 1
    a, b = g[-(first + n)], g[-first]
    seg = rows[a + 1:b + 1]
    span = int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])
    tot = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in seg:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy += d
        k = r["Kernel_Name"][:60] + " g=" + r["Grid_Size_X"] + "x" + r["Grid_Size_Y"] + "x" + r["Grid_Size_Z"]
        tot[k][0] += 1
        tot[k][1] += d
    print(f"per step: span {span / n / 1e3:.1f} us, busy {busy / n / 1e3:.1f} us, launches {len(seg) / n:.1f}")
    for k, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:85s} {c / n:6.1f}/step {d / n / 1e3:8.1f} us/step {d / c / 1e3:7.2f} us avg")


if __name__ == "__main__":
    main()
