#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_dac_gpu.py tests/test_kokoro_gpu.py tests/test_conv_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?
grep -E "max err|passed|failed|FAIL" gpurun_out/pytest_conv.log | tail -30
for a in; do
timeout -k 10 200 python3 bench.py --steps 200 --warmup 3 --no-cpu-baseline --orpheus-steps 0 --dia-steps 0 --conv-acc $a > gpurun_out/conv_b_$a.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/conv_b_$a.log').read().strip().splitlines()[-1]); print('acc $a value', d['value'], 'dac', d['dac_audio_sec_per_s'], 'kokoro', d['kokoro']['audio_sec_per_s'])"
done
exit $rc
