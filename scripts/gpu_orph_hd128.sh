#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_orpheus_gpu.py > gpurun_out/h128.log 2>&1
rc=$?
tail -2 gpurun_out/h128.log
exit $rc
