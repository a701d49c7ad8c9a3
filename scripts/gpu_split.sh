#!/bin/bash
# split codec convolutions: parity (DAC, Kokoro, SNAC, conv ops) and DAC timing at short / long lengths
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dac_gpu.py tests/test_conv_gpu.py tests/test_snac_gpu.py tests/test_kokoro_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_split.log 2>&1 || { tail -30 gpurun_out/t_split.log; exit 1; }
tail -1 gpurun_out/t_split.log
timeout -k 10 300 python3 scripts/bench_dac.py 20 100 861 > gpurun_out/dac_split.jsonl 2>&1 || { cat gpurun_out/dac_split.jsonl; exit 1; }
cat gpurun_out/dac_split.jsonl
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --orpheus-steps 0 --dia-steps 0 --kokoro-prompts 0 > gpurun_out/b_split.log 2>&1 || exit 1
tail -1 gpurun_out/b_split.log | cut -c1-330
