#!/bin/bash
# Round 6: per-layer kernel timeline of the 8-prompt step (one replica, one stream), the bench trace with
# packet capture off, then the tracer repro (packet capture on, crash handler) once.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl8 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 \
  --prompts 8 --replicas 1 --p8 0 --no-dac --no-cpu-baseline --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 \
  --sampled-steps 0 --prompt-pass 0 > gpurun_out/tl8.log 2>&1
rc=$?; echo "tl8 rc $rc"; tail -c 400 gpurun_out/tl8.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tl8 -name "*kernel_trace.csv" | head -1)
python3 scripts/step_timeline.py "$f" k_embed_sum -v > gpurun_out/tl8_step.txt; tail -30 gpurun_out/tl8_step.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl64 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 \
  --prompts 32 --replicas 1 --p8 0 --no-dac --no-cpu-baseline --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 \
  --sampled-steps 0 --prompt-pass 0 > gpurun_out/tl32.log 2>&1
rc=$?; echo "tl32 rc $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tl64 -name "*kernel_trace.csv" | head -1)
python3 scripts/step_timeline.py "$f" k_embed_sum -v > gpurun_out/tl32_step.txt; tail -30 gpurun_out/tl32_step.txt
unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
bash scripts/gpu_trace_r6.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_tracer_repro.sh
