#!/bin/bash
# Replicas per GPU for the lock-step AR step: 2 x 32 vs 3 x 22 (per-prompt rate), interleaved blocks per run.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/ab_ar.py --prompts 64 --replicas 2 --blocks 5 --steps 12 base= > gpurun_out/r6s_r2.log 2>&1 &&
timeout -k 10 300 python3 -u scripts/ab_ar.py --prompts 66 --replicas 3 --blocks 5 --steps 12 base= > gpurun_out/r6s_r3.log 2>&1 &&
timeout -k 10 300 python3 -u scripts/ab_ar.py --prompts 64 --replicas 2 --blocks 5 --steps 12 base= > gpurun_out/r6s_r2b.log 2>&1
rc=$?; grep variant gpurun_out/r6s_*.log; exit $rc
