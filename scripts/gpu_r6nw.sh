#!/bin/bash
# Prefill GEMM with 8 waves per workgroup: parity, then the batched prompt pass A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gemv_gpu.py -k "gemm_pf" > gpurun_out/r6nw_gemv.log 2>&1
rc=$?; tail -3 gpurun_out/r6nw_gemv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 2 nw4=GEMM_PF_NW:4 nw8=GEMM_PF_NW:8 > gpurun_out/r6nw_pp.log 2>&1
rc=$?; cat gpurun_out/r6nw_pp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 1 nw4=GEMM_PF_NW:4 nw8=GEMM_PF_NW:8 > gpurun_out/r6nw_pp1.log 2>&1
rc=$?; cat gpurun_out/r6nw_pp1.log; exit $rc
