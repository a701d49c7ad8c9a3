#!/bin/bash
# A/B of the split-scores chunk (ATTN_KS) at a long KV, then the tracer repro over 80 steps that cross no
# attention-kernel boundary (KV 600 -> 685)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/ab_ar.py --ctx 1100 ks2=ATTN_KS:2 ks4=ATTN_KS:4 ks1=ATTN_KS:1 > gpurun_out/ab_ks.log 2>&1 || { tail -5 gpurun_out/ab_ks.log; exit 1; }
grep '^{' gpurun_out/ab_ks.log | cut -c1-160
for rp in 2 4 2 4; do
  timeout -k 10 300 python3 scripts/ab_ar.py --ctx 448 --blocks 3 --replicas $rp a=ATTN_KS:2 > gpurun_out/ab_r$rp.log 2>&1 || { tail -5 gpurun_out/ab_r$rp.log; exit 1; }
  grep '^{' gpurun_out/ab_r$rp.log | cut -c1-160
done
TRACER_FULL=1 TRACER_EXTRA="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 --b1-replicas 0 --steps 80 --ctx 600" bash scripts/gpu_tracer_repro.sh
