#!/bin/bash
# The batched prompt pass's kernels (1 warm + 4 traced passes of 32 ragged prompts, packet capture off),
# then the streaming-copy variants (scripts/copy_peak.hip).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp_trace -o run --output-format csv -- python3 scripts/prompt_pass_probe.py 32 4 1 > gpurun_out/pp_trace.log 2>&1
rc=$?; echo "pp trace rc $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pp_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$f" k_gemv_q4K_kr k_attn k_bgemm > gpurun_out/pp_summary.txt; head -45 gpurun_out/pp_summary.txt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/copy_peak.hip -o gpurun_out/copy_peak 2>/dev/null &&
timeout -k 10 120 gpurun_out/copy_peak > gpurun_out/copy_peak.txt 2>&1; rc=$?; cat gpurun_out/copy_peak.txt; rm -f gpurun_out/copy_peak
exit $rc
