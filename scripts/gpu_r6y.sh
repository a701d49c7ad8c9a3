#!/bin/bash
# Multi-query short-context attention (k_attn_small_q): parity, runners' prompt passes, prompt-pass time.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_attn_gpu.py > gpurun_out/r6y_attn.log 2>&1
rc=$?; tail -3 gpurun_out/r6y_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parler_gpu.py tests/test_orpheus_gpu.py tests/test_dia_gpu.py tests/test_coalesce_gpu.py > gpurun_out/r6y_runners.log 2>&1
rc=$?; tail -3 gpurun_out/r6y_runners.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/prompt_pass_probe.py 32 6 2 > gpurun_out/r6y_pp.log 2>&1
rc=$?; cat gpurun_out/r6y_pp.log; [ $rc -eq 0 ] || exit $rc
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp_trace4 -o run --output-format csv -- python3 scripts/prompt_pass_probe.py 32 4 1 > gpurun_out/pp_trace4.log 2>&1
rc=$?; echo "pp trace rc $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pp_trace4 -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$f" k_attn > gpurun_out/pp_summary4.txt; head -20 gpurun_out/pp_summary4.txt; rm -f "$f"
