#!/bin/bash
# rocprofv3 kernel stats for the Kokoro generator bench (and optionally DAC): CSVs under gpurun_out/.
# usage (on the GPU box): bash scripts/gpu_prof_kokoro.sh [frames]
set -e
R=$GRAFT_REPO_ROOT
F=${1:-800}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kkprof -o kk --output-format csv -- python3 $R/scripts/bench_kokoro.py $F > $R/gpurun_out/kk_prof.log 2>&1
