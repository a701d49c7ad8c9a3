#!/bin/bash
# Development loop on the GPU box: parity tests, short bench, kernel-trace stats of the bench and
# of the GEMV micro-benchmark.  Every GPU step has its own time limit; the chain stops at the first
# failure.       gpurun -- bash scripts/gpu_iter.sh [bench args]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profg -o run --output-format csv -- python3 scripts/bench_gemv.py 20 > gpurun_out/profg.log 2>&1
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench.log | cut -c1-1500
for d in prof profg; do
  f=$(find gpurun_out/$d -name '*kernel_stats.csv' 2>/dev/null | head -1)
  [ -n "$f" ] && head -12 "$f" | cut -d, -f1-4
done
exit $rc
