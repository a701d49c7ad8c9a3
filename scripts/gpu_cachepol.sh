#!/bin/bash
# MALL-residency study: cache policy of the weight stream (nt / plain) and of the K/V stream (plain / nt),
# Parler AR decode (B = 8) and Orpheus decode, one build variant each (Makefile variant-%).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in "" wplain kvnt wplain_kvnt ""; do
  TTS_HIP_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 \
      --orpheus-steps 0 --dia-steps 0 > gpurun_out/cp_ar_$v.log 2>&1 || exit 1
  TTS_HIP_LIB_VARIANT=$v timeout -k 10 200 python3 scripts/bench_orpheus.py 8 64 32 > gpurun_out/cp_orph_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/cp_ar_$v.log').read().strip().splitlines()[-1])
o=json.loads(open('gpurun_out/cp_orph_$v.log').read().strip().splitlines()[-1])
print('variant [$v]', 'parler ar_ms_per_step', d['ar_ms_per_step'], 'gemv_us', d['roofline']['avg_launch_us'], '| orpheus ms_per_step', o['ms_per_step'])"
done
