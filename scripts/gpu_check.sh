#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprofv3 kernel stats.  Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?
echo "exit $rc"
tail -5 gpurun_out/pytest_gpu.log; tail -3 gpurun_out/smoke.log; tail -3 gpurun_out/bench.log
exit $rc
