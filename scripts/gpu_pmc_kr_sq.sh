#!/bin/bash
# SQ counters of the K-relay matrix-core Q4_K GEMV inside the Orpheus leg (8 prompts, M = 8): instruction
# mix (VALU : MFMA), wait and busy cycles per dispatch, grouped by template instance and grid (q/k/v, o,
# gate/up, down).  One --pmc pass of 8 SQ counters, kernel trace only; the last 896 dispatches are kept.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dac --graphs 0 --ctx 16 --kokoro-prompts 0 --dia-steps 0 --b1-replicas 0 --orpheus-steps 8"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-trace -d gpurun_out/pmc_krsq -o run --output-format csv -- $B > gpurun_out/pmc_krsq.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob, collections, json
fs = glob.glob("gpurun_out/pmc_krsq/**/*counter_collection.csv", recursive=True)
if not fs: raise SystemExit("no counter_collection.csv")
rows = [r for f in fs for r in csv.DictReader(open(f)) if "k_gemv_q4K_kr" in r["Kernel_Name"]]
disp = sorted({int(r["Dispatch_Id"]) for r in rows})[-896:]
keep = set(disp)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if int(r["Dispatch_Id"]) not in keep: continue
    k = r["Kernel_Name"].split("(")[0].split("<")[-1].rstrip(">") + " grid " + r["Grid_Size"]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in agg.items():
    m = {c: round(sum(v) / len(v)) for c, v in cs.items()}
    m["dispatches"] = len(next(iter(cs.values())))
    if m.get("SQ_INSTS_MFMA"): m["valu_per_mfma"] = round(m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"], 2)
    if m.get("SQ_WAVE_CYCLES"): m["wait_any_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
    out[k] = m
json.dump({"command": "rocprofv3 --pmc <8 SQ counters> --kernel-trace -- " + "bench.py Orpheus leg (scripts/gpu_pmc_kr_sq.sh)",
           "note": "per-dispatch averages over the last 896 k_gemv_q4K_kr dispatches (8 decode steps x 28 layers x 4 launches), M = 8",
           "kernels": out}, open("gpurun_out/pmc_kr_sq.json", "w"), indent=1)
for k, m in out.items(): print(k, m)
PY
exit $rc
