#!/bin/bash
# attention parity (eight-wave P.V), then AR studies: warmup length / idle gap, eight-wave P.V at KV 448 / 1200
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r4g
timeout -k 10 300 python -u -m pytest tests/test_attn_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4g/tests.log 2>&1 || { tail -20 gpurun_out/r4g/tests.log; exit 1; }
tail -1 gpurun_out/r4g/tests.log
NO_TESTS=1 VARIANTS="w50:--no-dac --warmup 50|w50idle:--no-dac --warmup 50 --idle-ms 500|w20:--no-dac --warmup 20|w5:--no-dac --warmup 5|mp2:--no-dac --warmup 50 --attn-pv-mp 2|mp1c:--no-dac --warmup 50 --ctx 1200|mp2c:--no-dac --warmup 50 --ctx 1200 --attn-pv-mp 2|nw8:--no-dac --warmup 50 --gemm-kr-nw 8" bash scripts/gpu_dacb.sh
