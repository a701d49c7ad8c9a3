#!/bin/bash
# Split P.V with the whole V slice requested before the softmax: attention parity, Parler AR A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_gpu.py tests/test_parler_gpu.py > gpurun_out/pv_tests.log 2>&1
rc=$?
tail -2 gpurun_out/pv_tests.log
[ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
timeout -k 10 200 python3 bench.py --steps 400 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 \
    --dia-steps 0 --attn-pv16 $v > gpurun_out/pv_ar_$v.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads(open('gpurun_out/pv_ar_$v.log').read().strip().splitlines()[-1])
print('pv16 $v', 'ar_ms_per_step', d['ar_ms_per_step'], 'ar', d['ar_audio_sec_per_s'])"
done
