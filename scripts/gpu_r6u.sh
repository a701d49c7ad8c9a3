#!/bin/bash
# The batched prompt pass's kernels with the prefill GEMM (1 warm + 4 traced passes, one replica).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp_trace2 -o run --output-format csv -- python3 scripts/prompt_pass_probe.py 32 4 1 > gpurun_out/pp_trace2.log 2>&1
rc=$?; echo "pp trace rc $rc"; grep "median\|host" gpurun_out/pp_trace2.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pp_trace2 -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$f" k_gemm_q4K_pf k_gemv_q4K_kr k_attn > gpurun_out/pp_summary2.txt; head -40 gpurun_out/pp_summary2.txt
