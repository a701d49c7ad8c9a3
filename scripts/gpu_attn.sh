#!/bin/bash
# Attention parity tests + split/unsplit micro-benchmark with kernel-trace stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_attn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profa -o run --output-format csv -- python3 scripts/bench_attn.py 30 > gpurun_out/bench_attn.log 2>&1
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pytest_attn.log; cat gpurun_out/bench_attn.log | grep '^{'
f=$(find gpurun_out/profa -name '*kernel_stats.csv' 2>/dev/null | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -12
exit $rc
