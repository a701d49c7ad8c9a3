#!/bin/bash
# Hoist buffer reused once earlier hoisted products are copied back (q / k / v grouped in every prompt-pass
# layer): the whole GPU suite, then the prompt pass.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6h2_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r6h2_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 2 > gpurun_out/r6h2_pp.log 2>&1
rc=$?; cat gpurun_out/r6h2_pp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 1 > gpurun_out/r6h2_pp1.log 2>&1
rc=$?; cat gpurun_out/r6h2_pp1.log; exit $rc
