#!/bin/bash
# DAC-44k decode throughput and kernel-trace stats.   gpurun -- bash scripts/gpu_prof_dac.sh [frames...]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
F="${@:-50 200 861}"
timeout -k 10 300 python3 scripts/bench_dac.py $F > gpurun_out/dac_bench.jsonl 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profd -o run --output-format csv -- python3 scripts/bench_dac.py 200 > gpurun_out/profd.log 2>&1
rc=$?
cat gpurun_out/dac_bench.jsonl
f=$(find gpurun_out/profd -name '*kernel_stats.csv' 2>/dev/null | head -1)
[ -n "$f" ] && head -25 "$f" | cut -d, -f1-4
exit $rc
