#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_dia_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_dia.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/pytest_dia.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 64 > gpurun_out/dia_bench.log 2>&1; rc=$?
tail -3 gpurun_out/dia_bench.log
exit $rc
