#!/bin/bash
# Kernel-trace statistics of the bench and of the GEMV micro-benchmark (no tests).
#   gpurun -- bash scripts/gpu_prof.sh [bench args]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profg -o run --output-format csv -- python3 scripts/bench_gemv.py 20 > gpurun_out/profg.log 2>&1
rc=$?
echo "exit $rc"
for d in prof profg; do
  f=$(find gpurun_out/$d -name '*kernel_stats.csv' 2>/dev/null | head -1)
  [ -n "$f" ] && head -14 "$f" | cut -d, -f1-4
done
exit $rc
