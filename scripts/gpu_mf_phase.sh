#!/bin/bash
# matrix-core GEMV phase study (tile-streaming kernel): dbg bits 1 skip rows, 2 skip prologue, 4 plain loads
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
S=orpheus_up,orpheus_down,orpheus_head,parler_qkvo
: > gpurun_out/gemv_phase.jsonl
for dbg in ${DBGS:-0 2 4 6}; do
  timeout -k 10 120 python3 scripts/bench_gemv.py 20 1,8 1 $S 0 $dbg >> gpurun_out/gemv_phase.jsonl 2>&1 || exit 1
done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/gemv_phase.jsonl") if l.startswith("{")]
for r in rows: print(r["shape"], "M", r["M"], "dbg", r["dbg"], r["avg_us"], r["GBps"])
PY
