#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/profd20 -o run --output-format csv -- python3 $R/scripts/bench_dac.py 20 > $R/gpurun_out/profd20.log 2>&1 || exit 1
