#!/bin/bash
# graph replay across kernel switches (parity), then the tracer with packet capture on over a headline run
# whose KV length crosses 512 (the step graph's attention grid changes mid-run)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parler_gpu.py tests/test_gemv_gpu.py -x -q -k "graph_replay or in_kernel" --timeout 300 --timeout-method thread > gpurun_out/replay_test.log 2>&1 || { tail -30 gpurun_out/replay_test.log; exit 1; }
tail -1 gpurun_out/replay_test.log
timeout -k 10 300 python3 scripts/ab_ar.py --ctx 448 a=GEMM_KR_INKERNEL:0 ink=GEMM_KR_INKERNEL:64 > gpurun_out/ab_ink.log 2>&1 || { tail -5 gpurun_out/ab_ink.log; exit 1; }
grep '^{' gpurun_out/ab_ink.log | cut -c1-160
# kernel trace of the short headline (batched DAC) with packet capture off
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4h_trace -o run --output-format csv -- python3 $R/bench.py --steps 20 --no-cpu-baseline --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 --p8 0 > $R/gpurun_out/r4h_trace.log 2>&1 || { echo "trace failed"; tail -5 $R/gpurun_out/r4h_trace.log; exit 1; }
echo "trace ok"
unset DEBUG_CLR_GRAPH_PACKET_CAPTURE; cd $R
TRACER_FULL=1 TRACER_EXTRA="${TRACER_EXTRA:---no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 --b1-replicas 0 --steps 80}" bash scripts/gpu_tracer_repro.sh
