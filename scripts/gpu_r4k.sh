#!/bin/bash
# DAC batching study: 861-frame default line (1 / 2 / 4 prompts per decode), then 8 prompts per GPU (the
# 8-GPU share) at 20 frames (1 / 2 / 4 / 8 prompts per decode)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
NO_TESTS=1 STEPS=861 VARIANTS="b1:--dac-batch 1|b2:--dac-batch 2|b4:--dac-batch 4" bash scripts/gpu_dacb.sh || exit 1
mkdir -p gpurun_out/dacb861 && cp gpurun_out/dacb/b1.log gpurun_out/dacb/b2.log gpurun_out/dacb/b4.log gpurun_out/dacb861/
NO_TESTS=1 STEPS=20 VARIANTS="p8b1:--prompts 8 --dac-batch 1|p8b2:--prompts 8 --dac-batch 2|p8b4:--prompts 8 --dac-batch 4|p8b8:--prompts 8 --dac-batch 8|p8b1r:--prompts 8 --dac-batch 1|p8b8r:--prompts 8 --dac-batch 8" bash scripts/gpu_dacb.sh
