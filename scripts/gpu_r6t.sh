#!/bin/bash
# Prefill GEMM (k_gemm_q4K_pf): parity of every many-column Q4_K path, the runners' prompt passes, then
# the batched prompt pass A/B (K-relay GEMM vs prefill GEMM).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gemv_gpu.py -k "prefill or many" > gpurun_out/r6t_gemv.log 2>&1
rc=$?; tail -3 gpurun_out/r6t_gemv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parler_gpu.py tests/test_orpheus_gpu.py > gpurun_out/r6t_runners.log 2>&1
rc=$?; tail -3 gpurun_out/r6t_runners.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 2 kr=GEMM_PF:0 pf=GEMM_PF:64 > gpurun_out/r6t_pp.log 2>&1
rc=$?; cat gpurun_out/r6t_pp.log; exit $rc
