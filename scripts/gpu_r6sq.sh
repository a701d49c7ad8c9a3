#!/bin/bash
# k_attn_small_q with 16 waves per workgroup: attention + runner parity, then the prompt pass.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_attn_gpu.py > gpurun_out/r6sq_attn.log 2>&1
rc=$?; tail -2 gpurun_out/r6sq_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parler_gpu.py tests/test_coalesce_gpu.py > gpurun_out/r6sq_runners.log 2>&1
rc=$?; tail -2 gpurun_out/r6sq_runners.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 2 > gpurun_out/r6sq_pp.log 2>&1
rc=$?; cat gpurun_out/r6sq_pp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 1 > gpurun_out/r6sq_pp1.log 2>&1
rc=$?; cat gpurun_out/r6sq_pp1.log; exit $rc
