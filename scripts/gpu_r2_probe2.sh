#!/bin/bash
# round-2 probe 2: kernel trace of a 20-frame DAC decode (both conv_transpose paths)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profd20 -o run --output-format csv -- python3 $R/scripts/bench_dac.py 20 > $R/gpurun_out/profd20.log 2>&1 || exit 1
cd $R
cat gpurun_out/profd20.log | grep frames
