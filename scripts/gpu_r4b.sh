#!/bin/bash
# Round 4: GEMV parity after the XCD renumbering, then the driver's bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4b; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gemv_gpu.py tests/test_parler_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-3000
