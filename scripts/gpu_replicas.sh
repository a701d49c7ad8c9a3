#!/bin/bash
# AR step time vs concurrent replicas (8 prompts per GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for R in 1 2 4 8; do
  timeout -k 10 200 python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --replicas $R > gpurun_out/b_rep$R.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/b_rep$R.log').read().strip().splitlines()[-1]); print('replicas $R', d['ar_ms_per_step'], 'ms/step', d['ar_audio_sec_per_s'], 'audio-s/s')"
done
