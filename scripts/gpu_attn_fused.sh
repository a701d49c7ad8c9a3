#!/bin/bash
# One-launch decode attention: parity (attention tests, Parler tokens), micro-benchmark with kernel
# stats (rows / split / fused), Parler AR decode with the fused kernel on and off.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_gpu.py tests/test_parler_gpu.py > gpurun_out/af_tests.log 2>&1
rc=$?
tail -3 gpurun_out/af_tests.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profaf -o run --output-format csv -- python3 $R/scripts/bench_attn.py 30 > $R/gpurun_out/af_bench_attn.log 2>&1 || exit 1
cd $R
grep '^{' gpurun_out/af_bench_attn.log | cut -c1-200
f=$(find gpurun_out/profaf -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | grep -i attn
for af in 128 0; do
timeout -k 10 200 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 \
    --dia-steps 0 --attn-fused $af > gpurun_out/af_ar_$af.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads(open('gpurun_out/af_ar_$af.log').read().strip().splitlines()[-1])
print('attn_fused $af', 'ar_ms_per_step', d['ar_ms_per_step'], 'ar', d['ar_audio_sec_per_s'])"
done
