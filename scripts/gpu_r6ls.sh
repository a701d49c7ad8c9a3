#!/bin/bash
# Lock-step reference points for the B = 1 legs: one replica of 8 and one of 32 prompts at KV 448.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/ab_ar.py --prompts 8 --replicas 1 --blocks 4 --steps 12 base= > gpurun_out/r6ls_8.log 2>&1 &&
timeout -k 10 300 python3 -u scripts/ab_ar.py --prompts 32 --replicas 1 --blocks 4 --steps 12 base= > gpurun_out/r6ls_32.log 2>&1
rc=$?; grep variant gpurun_out/r6ls_*.log; exit $rc
