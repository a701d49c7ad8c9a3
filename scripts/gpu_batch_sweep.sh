#!/bin/bash
# AR-only throughput vs prompts per GPU and concurrent replicas
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for cfg in "8 2" "16 2" "16 4" "32 4" "64 4" "64 8"; do
  set -- $cfg
  timeout -k 10 150 python3 bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-dac --kokoro-prompts 0 --batch $1 --replicas $2 > gpurun_out/sweep_$1_$2.log 2>&1 || { echo "fail $cfg"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$1_$2.log').read().strip().splitlines()[-1]); print('$1 $2', d['value'], d['ar_ms_per_step'], d['roofline']['avg_launch_us'], d['host_us_per_step'])"
done
