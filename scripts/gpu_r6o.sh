#!/bin/bash
# Prompt-pass GEMM with row-tile walkers: parity, then interleaved A/B of the batched prompt pass.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemv_gpu.py -k "row_walk" > gpurun_out/r6o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6o_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 2 base=GEMM_KR_WALK:0 w4=GEMM_KR_WALK:4 w8=GEMM_KR_WALK:8 w16=GEMM_KR_WALK:16 > gpurun_out/r6o_pp.log 2>&1
rc=$?; cat gpurun_out/r6o_pp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 1 base=GEMM_KR_WALK:0 w4=GEMM_KR_WALK:4 w8=GEMM_KR_WALK:8 w16=GEMM_KR_WALK:16 > gpurun_out/r6o_pp1.log 2>&1
rc=$?; cat gpurun_out/r6o_pp1.log; exit $rc
