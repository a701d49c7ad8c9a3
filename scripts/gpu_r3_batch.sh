#!/bin/bash
# Round-3 batch: new kernels' parity (Q8_0 GEMM, batched f32 GEMM, sampler), reference-order runners,
# Dia full depth, then a short bench with the Dia encoder time.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
T="-x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gemv_gpu.py tests/test_ops_gpu.py tests/test_sampler_gpu.py tests/test_sampling_runners_gpu.py $T > gpurun_out/r3/kernels.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r3/kernels.log | head -30; exit 1; }
tail -1 gpurun_out/r3/kernels.log
timeout -k 10 500 python -u -m pytest tests/test_parler_gpu.py tests/test_orpheus_gpu.py tests/test_fusion_gpu.py $T > gpurun_out/r3/runners.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r3/runners.log | head -30; exit 1; }
tail -1 gpurun_out/r3/runners.log
timeout -k 10 500 python -u -m pytest tests/test_dia_gpu.py -s $T > gpurun_out/r3/dia.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r3/dia.log | head -30; exit 1; }
tail -1 gpurun_out/r3/dia.log
timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline --kokoro-prompts 0 --orpheus-steps 16 --b1-replicas 8 --b1-steps 50 > gpurun_out/r3/bench_short.log 2>&1 || { tail -5 gpurun_out/r3/bench_short.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r3/bench_short.log').read().strip().splitlines()[-1]);print(d['value'], d['ar_ms_per_step'], d['dia'], d['parler_b1'], d['orpheus']['ms_per_step'])"
