#!/bin/bash
# 64-prompt option study: replicas, xattn fusion, DAC workers
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
OPTS="r2:--replicas 2|r1:--replicas 1|r4:--replicas 4|r2_noxattn:--replicas 2 --fusion-mask 14335|r1_noxattn:--replicas 1 --fusion-mask 14335" STEPS=40 bash scripts/gpu_b64_opts.sh || exit 1
O=$R/gpurun_out/b64opts
for w in 8 16; do
  timeout -k 10 300 python3 bench.py --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --p8 0 --steps 20 --dac-workers $w > $O/dac_w$w.log 2>&1 || { tail -3 $O/dac_w$w.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('dac workers', sys.argv[2], 'value', d['value'], 'ar', d['ar_audio_sec_per_s'], 'dac', d['dac_audio_sec_per_s'])" $O/dac_w$w.log $w
done
