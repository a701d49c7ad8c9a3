#!/bin/bash
# Round 6 kernel trace of the driver's short bench line (AR + DAC of 20 frames, Kokoro / Orpheus / Dia legs;
# the 32-runner B=1 leg left out): rocprofv3 --kernel-trace --stats, with the runtime's graph-packet capture OFF
# (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0). With it on, the profiler's interception of hipGraphLaunch faulted on the host
# (profiles/r06/tracer_capture_on_bench20_segv.log); the kernels and their durations are the same.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace6 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --b1-wide 0 --sampled-steps 0 > gpurun_out/trace6.log 2>&1
rc=$?; echo "trace rc $rc"; tail -c 600 gpurun_out/trace6.log
f=$(find gpurun_out/trace6 -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/prof_summary.py "$f" k_gemv_q4K_kr k_attn_scores k_attn_pv_mp > gpurun_out/trace6_summary.txt && head -40 gpurun_out/trace6_summary.txt
exit $rc
