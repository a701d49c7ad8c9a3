#!/bin/bash
# Bench only (+ optional rocprof stats).  Usage: gpu_bench.sh [prof] [bench args...]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$1" = "prof" ]; then
  shift
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof.log 2>&1
else
  timeout -k 10 600 python3 bench.py "$@" > gpurun_out/bench.log 2>&1
fi
rc=$?
tail -2 gpurun_out/bench.log gpurun_out/prof.log 2>/dev/null | cut -c1-3000
exit $rc
