#!/bin/bash
# replica concurrency vs HIP hardware queues (AR only, 8 prompts per GPU)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for q in 4 8 16; do for cfg in "8 1" "8 2" "8 4"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python3 bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-dac --kokoro-prompts 0 --batch $1 --replicas $2 > gpurun_out/q_${q}_$2.log 2>&1 || { tail -5 gpurun_out/q_${q}_$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/q_${q}_$2.log').read().strip().splitlines()[-1]); print('queues $q replicas $2', d['value'], d['ar_ms_per_step'])"
done; done
