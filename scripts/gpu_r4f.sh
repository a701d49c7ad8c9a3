#!/bin/bash
# Orpheus PMC, then the 64-prompt option study (replicas, eight-wave GEMM, xattn fusion, DAC workers / split)
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/round
bash scripts/gpu_pmc_orpheus.sh > gpurun_out/round/pmc_orpheus.log 2>&1 || { tail -3 gpurun_out/round/pmc_orpheus.log; exit 1; }
OPTS="r2:--replicas 2|r2_nw8:--replicas 2 --gemm-kr-nw 8|r1:--replicas 1|r2_noxattn:--replicas 2 --fusion-mask 14335" STEPS=40 timeout -k 10 600 bash scripts/gpu_b64_opts.sh || exit 1
O=$R/gpurun_out/b64opts
for v in "w8:--dac-workers 8" "w16:--dac-workers 16" "w4:--dac-workers 4" "split256:--dac-conv-split 256" "split0:--dac-conv-split 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python3 bench.py --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --p8 0 --steps 20 $f > $O/dac_$n.log 2>&1 || { tail -3 $O/dac_$n.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('dac', sys.argv[2], 'value', d['value'], 'ar', d['ar_audio_sec_per_s'], 'dac', d['dac_audio_sec_per_s'])" $O/dac_$n.log $n
done
