#!/bin/bash
# Phase study of the lane-layout Q4_K GEMVs on Parler shapes, warm and cold caches.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 scripts/bin/gemv_phase > gpurun_out/parler_phase_warm.jsonl 2>&1 &&
GEMV_PHASE_COLD=1 timeout -k 10 120 scripts/bin/gemv_phase > gpurun_out/parler_phase_cold.jsonl 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("warm", "cold"):
    for l in open(f"gpurun_out/parler_phase_{f}.jsonl"):
        if not l.startswith("{"): print(l.strip()); continue
        x = json.loads(l)
        print(f, x["shape"], {k: x[k] for k in ("event_us", "chain_us", "span_us", "issue_us", "prologue_us", "barrier_us", "rows_us", "wait_w_us", "compute_us", "store_exit_us", "end_spread_us")})
PY
