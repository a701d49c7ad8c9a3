#!/bin/bash
# SQ counters of the matrix-core GEMV on Orpheus shapes (phase micro-benchmark, cold caches), two passes.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GEMV_PHASE_ORPHEUS=1 GEMV_PHASE_TILED=1 GEMV_PHASE_COLD=1 GEMV_KS=0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/pmco1 -o run --output-format csv -- ./scripts/bin/gemv_phase > gpurun_out/pmco1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES --kernel-trace -d gpurun_out/pmco2 -o run --output-format csv -- ./scripts/bin/gemv_phase > gpurun_out/pmco2.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob, collections
for d in ("pmco1", "pmco2"):
    fs = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)
    if not fs: print("no", d); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        if "q4K_mf" not in r["Kernel_Name"]: continue
        k = (r["Kernel_Name"].split("<")[-1].split(">")[0], r["Grid_Size"])
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        print(d, k, {c: round(sum(v) / len(v)) for c, v in cs.items()})
PY
exit $rc
