#!/bin/bash
# Kokoro end-to-end parity on the GPU (+ the generator's, whose uv/noise moved onto the device),
# then end-to-end throughput and a kernel trace of one 64-token run
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_lstm_gpu.py tests/test_fusion_gpu.py tests/test_kokoro_model_gpu.py tests/test_kokoro_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_kokoro.log 2>&1 || { tail -40 gpurun_out/t_kokoro.log; exit 1; }
grep -E "kokoro |passed|failed|FAIL" gpurun_out/t_kokoro.log
timeout -k 10 200 python -u scripts/bench_kokoro_model.py 16 64 > gpurun_out/b_kokoro_model.log 2>&1 || { tail -30 gpurun_out/b_kokoro_model.log; exit 1; }
cat gpurun_out/b_kokoro_model.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kokoro_model -o run --output-format csv -- python3 $R/scripts/bench_kokoro_model.py 64 > $R/gpurun_out/prof_kokoro_model.log 2>&1 || exit 1
find $R/gpurun_out/prof_kokoro_model -name "*kernel_stats.csv" | head -1 | xargs head -25
