#!/bin/bash
# Kernel trace of ONE DAC-44k decoder over a short clip (default 20 frames): per-shape kernel times
# of a single decode (the driver's short line runs 8 of these concurrently).
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/study
mkdir -p "$O"
F=${1:-20}
timeout -k 10 120 python3 "$R/scripts/bench_dac.py" $F --default-only > "$O/dac1.jsonl" 2>&1 &&
(cd /tmp && export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/profd1" -o run --output-format csv -- python3 "$R/scripts/bench_dac.py" $F --default-only > "$O/dac1_trace.log" 2>&1) &&
cat "$O/dac1.jsonl"
