#!/bin/bash
# Kokoro F16 (configs[1]) parity + conv_transpose F16 + the Kokoro bench leg alone.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kokoro_model_gpu.py tests/test_conv_gpu.py tests/test_kokoro_gpu.py tests/test_lstm_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3/k16_tests.log 2>&1 || { tail -30 gpurun_out/r3/k16_tests.log; exit 1; }
tail -3 gpurun_out/r3/k16_tests.log
timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline --orpheus-steps 0 --dia-steps 0 --no-dac > gpurun_out/r3/k16_bench.log 2>&1 || { tail -5 gpurun_out/r3/k16_bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r3/k16_bench.log').read().strip().splitlines()[-1]);print(json.dumps(d['kokoro']))"
