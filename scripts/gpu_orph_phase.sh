#!/bin/bash
# Phase study of the matrix-core GEMV on Orpheus shapes (cold caches), depth 2 vs 4, K-split off.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for d in 2; do
GEMV_PHASE_ORPHEUS=1 GEMV_PHASE_TILED=1 GEMV_PHASE_COLD=1 GEMV_KS=${KS:-0} timeout -k 10 120 scripts/bin/gemv_phase > gpurun_out/orph_phase_d$d.jsonl 2>&1 || exit 1
done
python3 - <<'PY'
import json
for d in (2,):
    for l in open(f"gpurun_out/orph_phase_d{d}.jsonl"):
        if not l.startswith("{"): print(l.strip()); continue
        x = json.loads(l)
        print(d, x["shape"], {k: x[k] for k in ("event_us", "chain_us", "span_us", "start_spread_us", "issue_us", "prologue_us", "barrier_us", "rows_us", "end_spread_us")})
PY
