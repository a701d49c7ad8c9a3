#!/bin/bash
# codec quantizer gather fusion: DAC / SNAC / Dia / adapter parity, then the short headline (twice)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r4m
timeout -k 10 600 python -u -m pytest tests/test_dac_gpu.py tests/test_snac_gpu.py tests/test_dia_gpu.py tests/test_adapter_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m/tests.log 2>&1 || { tail -30 gpurun_out/r4m/tests.log; exit 1; }
tail -1 gpurun_out/r4m/tests.log
NO_TESTS=1 VARIANTS="g1:--dac-batch 8|g2:--dac-batch 8" bash scripts/gpu_dacb.sh
