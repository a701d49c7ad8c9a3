#!/bin/bash
# unique-load GEMV: parity tests, phase timelines (both kernels), AR bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemv_gpu.py tests/test_fusion_gpu.py tests/test_parler_gpu.py tests/test_orpheus_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_u.log 2>&1 || { tail -30 gpurun_out/t_u.log; exit 1; }
tail -2 gpurun_out/t_u.log
for u in 0 1; do
  GEMV_UNIQUE=$u GEMV_PHASE_COLD=1 timeout -k 10 120 scripts/bin/gemv_phase > gpurun_out/phase_u$u.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/phase_u$u.jsonl'):
    d=json.loads(l); print('u=$u', d['shape'], 'span', d['span_us'], 'issue', d['issue_us'], 'pro', d['prologue_us'], 'bar', d['barrier_us'], 'rows', d['rows_us'])"
done
for u in 0 1; do
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --gemv-unique $u > gpurun_out/b_u$u.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/b_u$u.log').read().strip().splitlines()[-1]); print('u=$u', d['ar_ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['achieved'])"
done
