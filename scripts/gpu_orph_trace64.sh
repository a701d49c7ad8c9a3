#!/bin/bash
# in-graph per-kernel durations of the Orpheus decode step (B=8)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tro64 -o tr --output-format csv -- python3 $R/scripts/bench_orpheus.py 8 64 32 > $R/gpurun_out/tro64.log 2>&1 || exit 1
f=$(find $R/gpurun_out/tro64 -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/step_breakdown.py $f 10 10 9984 > $R/gpurun_out/tro64.txt
tail -1 $R/gpurun_out/tro64.log | cut -c1-300
head -24 $R/gpurun_out/tro64.txt
