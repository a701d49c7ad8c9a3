#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for u in 0 1; do
GEMV_UNIQUE=$u GEMV_PHASE_COLD=1 timeout -k 10 120 scripts/bin/gemv_phase > gpurun_out/phase_u$u.jsonl 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/phase_u$u.jsonl'):
    d=json.loads(l); print('u=$u', d['shape'], 'span', d['span_us'], 'issue', d['issue_us'], 'pro', d['prologue_us'], 'bar', d['barrier_us'], 'rows', d['rows_us'], 't34', d['t34_us'], 't45', d['t45_us'])"
done
