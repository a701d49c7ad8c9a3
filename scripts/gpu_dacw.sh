#!/bin/bash
# A/B of the concurrent DAC decoders on the driver's bench line (steps 20)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for w in 2 4 8; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --dac-workers $w > gpurun_out/b_dacw$w.log 2>&1 || exit 1
  echo "workers $w: $(tail -1 gpurun_out/b_dacw$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ar_audio_sec_per_s"], d["dac_audio_sec_per_s"])')"
done
