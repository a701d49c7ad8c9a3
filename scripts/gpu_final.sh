#!/bin/bash
# final round-4 lines on the final tree: GPU suite, smoke, default bench, the driver's short bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/final; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python3 bench.py > $O/bench_full.log 2>&1 &&
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -5 $O/pytest_gpu.log $O/smoke.log $O/bench_full.log $O/bench20.log; exit 1; }
tail -1 $O/pytest_gpu.log; tail -1 $O/smoke.log
tail -1 $O/bench20.log | cut -c1-300
