#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rocm-smi --showclocks > gpurun_out/clocks_before.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profg -o run --output-format csv -- python3 scripts/bench_gemv.py 20 > gpurun_out/profg.log 2>&1
rc=$?
rocm-smi --showclocks > gpurun_out/clocks_after.txt 2>&1 || true
exit $rc
