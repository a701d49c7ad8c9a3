#!/bin/bash
# kernel trace of AR decode only (1 replica, B prompts), summarised per kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
B=${1:-8}; CTX=${2:-448}; shift 2 2>/dev/null
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/arprof -o ar --output-format csv -- python3 $R/bench.py --steps 40 --warmup 2 --no-cpu-baseline --no-dac --kokoro-prompts 0 --batch $B --replicas 1 --ctx $CTX "$@" > $R/gpurun_out/ar_prof.log 2>&1
rc=$?
cd $R
tail -1 gpurun_out/ar_prof.log | cut -c1-600
f=$(find gpurun_out/arprof -name '*kernel_trace.csv' | head -1)
python3 scripts/step_breakdown.py $f 12 30 > gpurun_out/ar_prof_summary.txt
cat gpurun_out/ar_prof_summary.txt | head -40
exit $rc
