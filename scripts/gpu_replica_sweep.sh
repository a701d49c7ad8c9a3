#!/bin/bash
# Parler AR decode, 8 prompts per GPU: runner replicas 1 / 2 / 4 / 8 (each its own backend + stream).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for rep in 2 4 8 1; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 \
      --dia-steps 0 --replicas $rep > gpurun_out/rs_$rep.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/rs_$rep.log').read().strip().splitlines()[-1])
print('replicas $rep', 'ar_ms_per_step', d['ar_ms_per_step'], 'ar', d['ar_audio_sec_per_s'])"
done
for q in 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 \
      --dia-steps 0 --replicas 4 > gpurun_out/rs_q$q.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/rs_q$q.log').read().strip().splitlines()[-1])
print('queues $q replicas 4', 'ar_ms_per_step', d['ar_ms_per_step'], 'ar', d['ar_audio_sec_per_s'])"
done
