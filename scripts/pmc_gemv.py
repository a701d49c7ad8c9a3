#!/usr/bin/env python3
"""Fold two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM traffic of the
dominant kernel and write profiles/<round>/pmc_gemv_q4k.json, which bench.py reports as
roofline.traffic.

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE is in KiB and on gfx950 counts half
the bytes of 16-B-per-lane coalesced streaming reads (the Q4_K weight stream is exactly that), so it
is doubled; WRITE_SIZE is taken as reported.

Only the decode-step dispatches the bench's own roofline samples are kept: the last N launches of
the kernel, N = roofline.launches_sampled of the bench line in FETCH_DIR/../pmc_fetch.log.

usage: pmc_gemv.py FETCH_DIR WRITE_DIR OUT_JSON [kernel-substring [last-N [command]]]
(an explicit last-N replaces the bench line's launches_sampled, e.g. for the Orpheus leg)
"""
import csv
import glob
import json
import sys


def per_kernel(d, counter, pat, last):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and pat in r.get("Kernel_Name", ""):
                rows.append(r)
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    rows = rows[-last:]
    # key each launch by its position within the decode step (the period of the launch sequence), so
    # different matrices with one template / grid (Orpheus q / o / down) stay apart
    sig = [(r["Kernel_Name"], r["Grid_Size"]) for r in rows]
    period = len(sig)
    for p in range(1, len(sig) // 2 + 1):
        if all(sig[i] == sig[i - p] for i in range(p, len(sig))):
            period = p
            break
    shapes = {}
    for i, r in enumerate(rows):
        k = f'step pos {i % period:03d}: {r["Kernel_Name"].split("<")[-1].split(">")[0]} grid {r["Grid_Size"]}'
        shapes.setdefault(k, []).append(float(r["Counter_Value"]))
    return sum(float(r["Counter_Value"]) for r in rows), len(rows), shapes


def sampled_launches(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return int(json.loads(line)["roofline"]["launches_sampled"])
    raise SystemExit(f"no bench line in {log}")


def main():
    fdir, wdir, out = sys.argv[1:4]
    pat = sys.argv[4] if len(sys.argv) > 4 else "k_gemv_q4_K"
    last = int(sys.argv[5]) if len(sys.argv) > 5 else sampled_launches(fdir.rstrip("/") + ".log")
    cmd = sys.argv[6] if len(sys.argv) > 6 else (
        "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace --stats -- python3 bench.py --steps 10 "
        "--warmup 2 --no-cpu-baseline --no-dac --graphs 0 --ctx 16 (decode dispatches only)")
    f, nf, fs = per_kernel(fdir, "FETCH_SIZE", pat, last)
    w, nw, ws = per_kernel(wdir, "WRITE_SIZE", pat, last)
    if not nf or not nw:
        raise SystemExit(f"kernel {pat!r} not found (fetch {nf}, write {nw})")
    fetch = 2.0 * 1024.0 * f / nf
    write = 1024.0 * w / nw
    res = {"kernel": pat, "dispatches_fetch_pass": nf, "dispatches_write_pass": nw,
           "fetch_bytes_per_launch_raw": 1024.0 * f / nf, "fetch_bytes_per_launch": fetch,
           "write_bytes_per_launch": write, "hbm_bytes_per_launch": round(fetch + write, 1),
           "per_shape_hbm_bytes": {k: round(2048.0 * sum(v) / len(v) + 1024.0 * sum(ws.get(k, [0])) / max(len(ws.get(k, [])), 1), 1)
                                   for k, v in fs.items()},
           "largest_launch_fetch_bytes_raw": max(1024.0 * sum(v) / len(v) for v in fs.values()),
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count of 16B/lane streaming reads); WRITE_SIZE KiB x1024; "
                         "check it on a launch of known weight bytes (largest_launch_fetch_bytes_raw: the Orpheus head, 271 MB)",
           "launches_kept": last, "command": cmd}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
