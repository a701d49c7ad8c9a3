#!/bin/bash
# Prefill GEMM v2 (operand tile in LDS, two row tiles per wave): parity, A/B, kernel summary.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gemv_gpu.py -k "prefill or many" > gpurun_out/r6v_gemv.log 2>&1
rc=$?; tail -3 gpurun_out/r6v_gemv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parler_gpu.py tests/test_orpheus_gpu.py > gpurun_out/r6v_runners.log 2>&1
rc=$?; tail -3 gpurun_out/r6v_runners.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 2 kr=GEMM_PF:0 pf=GEMM_PF:64 > gpurun_out/r6v_pp.log 2>&1
rc=$?; cat gpurun_out/r6v_pp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 1 kr=GEMM_PF:0 pf=GEMM_PF:64 > gpurun_out/r6v_pp1.log 2>&1
rc=$?; cat gpurun_out/r6v_pp1.log; [ $rc -eq 0 ] || exit $rc
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp_trace3 -o run --output-format csv -- python3 scripts/prompt_pass_probe.py 32 4 1 > gpurun_out/pp_trace3.log 2>&1
rc=$?; echo "pp trace rc $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pp_trace3 -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$f" k_gemm_q4K_pf k_gemv_q4K_kr > gpurun_out/pp_summary3.txt; head -30 gpurun_out/pp_summary3.txt; rm -f "$f"
