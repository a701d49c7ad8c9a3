#!/bin/bash
# Parler AR decode only (8 prompts, 2 replicas), 200 steps, twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 200 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 \
    --dia-steps 0 > gpurun_out/arq_$k.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads(open('gpurun_out/arq_$k.log').read().strip().splitlines()[-1])
print('ar_ms_per_step', d['ar_ms_per_step'], 'ar', d['ar_audio_sec_per_s'], 'gemv_us', d['roofline']['avg_launch_us'])"
done
