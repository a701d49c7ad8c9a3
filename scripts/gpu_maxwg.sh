#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parler_gpu.py > gpurun_out/mw_tests.log 2>&1 || { tail -3 gpurun_out/mw_tests.log; exit 1; }
for cap in 0 128 192 0 128; do
TTS_HIP_GEMV_MAXWG=$cap timeout -k 10 200 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 \
    --dia-steps 0 > gpurun_out/mw_$cap.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads(open('gpurun_out/mw_$cap.log').read().strip().splitlines()[-1])
print('cap $cap', 'ar_ms_per_step', d['ar_ms_per_step'], 'gemv_us', d['roofline']['avg_launch_us'])"
done
