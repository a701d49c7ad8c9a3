#!/bin/bash
# Orpheus runner parity (GPU vs oracle)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_orpheus_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_orpheus.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/pytest_orpheus.log | head -30
exit $rc
