#!/bin/bash
# Orpheus decode bench (graphs) + kernel trace of a shorter eager run
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 scripts/bench_orpheus.py ${1:-8} ${2:-64} 32 > gpurun_out/orpheus_bench.log 2>&1 || { tail -20 gpurun_out/orpheus_bench.log; exit 1; }
tail -1 gpurun_out/orpheus_bench.log
cd /tmp && export TMPDIR=/tmp
TTS_BENCH_GRAPHS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/orprof -o or --output-format csv -- python3 $R/scripts/bench_orpheus.py ${1:-8} 16 32 > $R/gpurun_out/orpheus_prof.log 2>&1
rc=$?
cd $R
f=$(find gpurun_out/orprof -name '*kernel_stats.csv' | head -1)
head -16 "$f" | cut -d, -f1-5
exit $rc
