#!/bin/bash
# The profiling half of scripts/gpu_round.sh on its own: kernel-trace stats of the short bench, then the
# PMC HBM-traffic passes.  Every GPU step has its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --orpheus-steps 16 --dia-steps 16 $PROF_ARGS > $R/gpurun_out/prof.log 2>&1 || exit 1
cd $R
unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 &&
bash scripts/gpu_pmc_orpheus.sh > gpurun_out/pmc_orpheus.log 2>&1
