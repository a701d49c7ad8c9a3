#!/bin/bash
# Round 4: adapter executed end to end, then the 64-prompt study.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4a; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_adapter_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/adapter.log 2>&1
rc=$?; tail -15 $O/adapter.log
[ $rc -eq 0 ] || exit $rc
DAC=1 bash scripts/gpu_b64.sh
