#!/bin/bash
# parity tests, then a short bench (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 200 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench.log | cut -c1-3000
exit $rc
