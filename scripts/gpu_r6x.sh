#!/bin/bash
# Final round-6 evidence: the driver's default bench line, then the whole GPU suite.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r6x_bench.json 2> gpurun_out/r6x_bench.err
rc=$?; echo "bench rc $rc"; tail -c 1500 gpurun_out/r6x_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6x_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r6x_suite.log; exit $rc
