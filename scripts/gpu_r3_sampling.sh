#!/bin/bash
# Seeded sampler (device vs host), runner-level sampled tokens, reference-order runners, Dia full depth.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 300 python -u -m pytest tests/test_sampler_gpu.py tests/test_sampling_runners_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3/sampling_tests.log 2>&1 || { tail -40 gpurun_out/r3/sampling_tests.log; exit 1; }
tail -3 gpurun_out/r3/sampling_tests.log
timeout -k 10 500 python -u -m pytest tests/test_parler_gpu.py tests/test_orpheus_gpu.py tests/test_fusion_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3/runners.log 2>&1 || { tail -40 gpurun_out/r3/runners.log; exit 1; }
tail -3 gpurun_out/r3/runners.log
timeout -k 10 500 python -u -m pytest tests/test_dia_gpu.py -x -v -s --timeout 450 --timeout-method thread > gpurun_out/r3/dia_full.log 2>&1 || { tail -30 gpurun_out/r3/dia_full.log; exit 1; }
tail -3 gpurun_out/r3/dia_full.log
