#!/bin/bash
# Kernel timeline of the coalesced B = 1 step (8 ragged runners), packet capture off.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/b1_trace -o run --output-format csv -- python3 scripts/b1_probe.py 8 30 1 > gpurun_out/b1_trace.log 2>&1
rc=$?; echo "b1 trace rc $rc"; grep '^{' gpurun_out/b1_trace.log | tail -c 600; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/b1_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/step_timeline.py "$f" k_embed_sum -v > gpurun_out/b1_step.txt; tail -30 gpurun_out/b1_step.txt
rm -f "$f"
